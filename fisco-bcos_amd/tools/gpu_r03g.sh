# the -m gpu suite, then short C2 and C2-SM2 bench lines (inv_pipe only in the secp trio kernel)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
for wl in c2 c2sm2; do
  timeout -k 10 120 python3 bench.py --workload $wl --steps 2000 --warmup 20 --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/b_$wl.json'));print('$wl', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4))"
done
timeout -k 10 60 fisco-bcos_amd/lib/invbench
