# Merkle check: hash/Merkle GPU parity tests, then the C1 legs (100k widths 2 / 16) and 1M / 16M timings
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_hash.py tests/test_gpu_verify.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_merkle.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/pytest_merkle.log | tail -30; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_merkle.log; exit $rc; }
timeout -k 10 120 python3 fisco-bcos_amd/tools/merkle_trace.py 100000
