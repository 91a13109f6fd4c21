# One GPU call: the -m gpu suite, then bench lines for every workload, then (optionally) profiles.
# Stops at the first step that times out / crashes (rc >= 124 or signal); test assertion failures
# (pytest rc 1) do not stop the benches.
# usage: bash fisco-bcos_amd/tools/gpu_round.sh "<workloads>" "<profile workloads>"
WLS=${1:-"c2"}; PROF=${2:-""}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for wl in $WLS; do
  steps=20; [ $wl = c3 ] || [ $wl = c4 ] || [ $wl = c5 ] && steps=5
  timeout -k 10 300 python3 bench.py --workload $wl --steps $steps --warmup 2 > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  r=$?; echo "bench $wl rc=$r"; tail -c 1500 gpurun_out/bench_$wl.json
  if [ $r -ne 0 ]; then tail -20 gpurun_out/bench_$wl.err; exit $r; fi
done
for wl in $PROF; do
  steps=10; [ $wl = c3 ] || [ $wl = c4 ] || [ $wl = c5 ] && steps=3
  bash fisco-bcos_amd/tools/gpu_profile.sh $wl $steps 240 || exit $?
done
exit 0
