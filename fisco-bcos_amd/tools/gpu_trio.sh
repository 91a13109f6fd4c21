# lane-trio kernel check: variant agreement + tx-verify parity, then the C2 bench with the trio and the pair kernels
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "variants or synthetic or ragged" > gpurun_out/pytest_trio.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/pytest_trio.log | tail -14; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_trio.log; exit $rc; }
for c in 2 1; do
  BCOSGPU_TXV_COOP=$c timeout -k 10 200 python3 bench.py --workload c2 --steps 2000 --warmup 3 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/bench_c2_coop$c.json 2> gpurun_out/bench_c2_coop$c.err || { tail -20 gpurun_out/bench_c2_coop$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_c2_coop$c.json'));print('coop=$c', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
