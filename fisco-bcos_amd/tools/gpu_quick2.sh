# secp parity (both fields, all variants) + C4 / C2 timing
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_q2.log | head; exit $rc; }
for wl in c4 c2; do
  timeout -k 10 200 python3 bench.py --workload $wl --steps 200 --warmup 5 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/q2_$wl.json 2> gpurun_out/q2_$wl.err || { tail -20 gpurun_out/q2_$wl.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/q2_$wl.json'));print('$wl', round(d['value']/1e6,3), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],4))"
done
