mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sm2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sm2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_sm2.log | head -20; exit $rc; }
for f in 1 0; do
  BCOSGPU_K1_F26=$f timeout -k 10 200 python3 bench.py --workload c2sm2 --steps 200 --warmup 20 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/sm2_c2.json 2> gpurun_out/sm2_c2.err || { tail -20 gpurun_out/sm2_c2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sm2_c2.json'));print('c2sm2 f26=$f', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],3), d['config'].get('kernel'))"
done
