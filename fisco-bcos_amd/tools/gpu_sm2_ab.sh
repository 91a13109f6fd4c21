# SM2 GPU tests at the tree, then the c2sm2 library A/B (lib_ab/libbcosgpu_A.so vs lib/)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ecc.py tests/test_gpu_verify.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_sm2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_sm2.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_sm2.log | head -30; exit $rc; }
bash fisco-bcos_amd/tools/gpu_lib_ab.sh c2sm2 3000
