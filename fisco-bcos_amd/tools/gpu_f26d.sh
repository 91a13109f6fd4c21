# fe26 everywhere: phases of the coop kernel, the secp GPU tests on both fields, C2 bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 100 fisco-bcos_amd/lib/coopbench 26 > gpurun_out/coop26_phases.json || exit 1
cat gpurun_out/coop26_phases.json
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_verify.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_f26d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -cE "PASSED" gpurun_out/pytest_f26d.log; grep -E "FAILED|Error" gpurun_out/pytest_f26d.log | tail -5; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_f26d.log; exit $rc; }
timeout -k 10 200 python3 bench.py --steps 1000 --warmup 20 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/bench_c2_f26d.json 2> gpurun_out/bench_c2_f26d.err || { tail -20 gpurun_out/bench_c2_f26d.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_c2_f26d.json'));print('c2', d['value'], d['roofline']['kernel_ms'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_hash.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_hash.log 2>&1 || { tail -30 gpurun_out/pytest_hash.log; exit 1; }
tail -2 gpurun_out/pytest_hash.log
timeout -k 10 300 python3 bench.py --steps 500 --warmup 20 --warm-seconds 1 --legs= --no-cpu-baseline --no-extras > gpurun_out/bench_merkle.json 2> gpurun_out/bench_merkle.err || { tail -20 gpurun_out/bench_merkle.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_merkle.json'))
m=d.get('merkle_c1') or d.get('merkle')
print(json.dumps(m)[:1500])"
