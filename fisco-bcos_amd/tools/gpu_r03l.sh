# Merkle node reads without per-word branches (NodeReader): hash GPU tests, the one-launch probe, and
# a C1 A/B of the one-launch and two-launch paths for both hashers
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 fisco-bcos_amd/lib/keccakpair_check > gpurun_out/keccakpair.json 2>&1 || { cat gpurun_out/keccakpair.json; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_hash.py tests/test_gpu_verify.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_hash.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_hash.log | head -30; exit $rc; }
timeout -k 10 60 fisco-bcos_amd/lib/fusedprobe | tee gpurun_out/fusedprobe2.log || exit 1
timeout -k 10 60 fisco-bcos_amd/lib/sm3probe | tee gpurun_out/sm3probe.log || exit 1
for i in 1 2; do for v in 0 1; do
  echo "fused=$v $(BCOSGPU_MERKLE_FUSED=$v timeout -k 10 60 python3 fisco-bcos_amd/tools/merkle_trace.py 100000 16 400 | tr '\n' ' ')" || exit 1
done; done 2>&1 | tee gpurun_out/merkle_noderead_ab.log
