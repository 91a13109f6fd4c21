# SM2 trio kernel with the Jacobian-entry windows: phase probe, the SM2 GPU tests, then a short c2sm2 bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 60 fisco-bcos_amd/lib/sm2bench || exit 1; done 2>&1 | tee gpurun_out/sm2_phases_jac.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_verify.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_sm2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sm2.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_sm2.log | head -30; exit $rc; }
for wl in c2sm2; do
  timeout -k 10 120 python3 bench.py --workload $wl --steps 2000 --warmup 20 --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/b_$wl.json'));print('$wl', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4))"
done
