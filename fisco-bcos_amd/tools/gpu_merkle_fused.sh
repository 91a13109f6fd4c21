# The one-launch Merkle path: hash latencies, the Merkle GPU parity tests, then an A/B of the
# fused path against the multi-launch path at C1 (100k leaves) and 1M leaves, widths 16 and 2.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 fisco-bcos_amd/lib/keccakpair_check > gpurun_out/hash_latency.json 2>&1
rc=$?; cat gpurun_out/hash_latency.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_hash.py tests/test_gpu_verify.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_hash.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_hash.log | head -30; exit $rc; }
for n in 100000 1000000; do for v in 0 1; do for w in 16 2; do
  echo "n=$n fused=$v w=$w $(BCOSGPU_MERKLE_FUSED=$v timeout -k 10 60 python3 fisco-bcos_amd/tools/merkle_trace.py $n $w 200 | tr '\n' ' ')" || exit 1
done; done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/merkle_fused_ab.log
