mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "variants or synthetic" > gpurun_out/pytest_pair.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/pytest_pair.log | tail -12; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_pair.log; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 500 --legs c2sm2 --no-merkle --no-cpu-baseline --no-extras > gpurun_out/bench_pair.json 2> gpurun_out/bench_pair.err
r=$?; echo "bench rc=$r"; tail -c 400 gpurun_out/bench_pair.err; exit $r
