mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
r=$?; echo "bench default rc=$r"; tail -c 600 gpurun_out/bench_default.err; [ $r -eq 0 ] || exit $r
BCOSGPU_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 300 --no-merkle --no-cpu-baseline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
r=$?; echo "bench gloo2 rc=$r"; tail -c 600 gpurun_out/bench_gloo2.err; exit $r
