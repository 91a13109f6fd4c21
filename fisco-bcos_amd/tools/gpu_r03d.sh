# Trio kernel phase-D A/B: phase timestamps of the previous builds (A: round-2 kernel, B1: pipelined
# inversion + comb rebalance) and the current one (trio additions + lane-pair address Keccak), then the
# full -m gpu suite and a C2-only bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in A B1; do echo "$v $(timeout -k 10 60 fisco-bcos_amd/lib_ab/coopbench_$v trio)" || exit 1; done
  echo "B2 $(timeout -k 10 60 fisco-bcos_amd/lib/coopbench trio)" || exit 1
done 2>&1 | tee gpurun_out/trio_phase_ab.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u bench.py --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; exit $rc
