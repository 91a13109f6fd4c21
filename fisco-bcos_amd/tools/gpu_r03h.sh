# zz window in the trio kernel: phase timestamps, the -m gpu suite, a C2 bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do echo "zz $(timeout -k 10 60 fisco-bcos_amd/lib/coopbench trio)" || exit 1; done | tee gpurun_out/trio_phase_zz.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 120 python3 bench.py --workload c2 --steps 2000 --warmup 20 --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/b_c2.json'));print('c2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4))"
