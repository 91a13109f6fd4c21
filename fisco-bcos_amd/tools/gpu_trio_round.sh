# the -m gpu suite, the C2 profile (kernel trace + PMC passes) and the default bench line, one call
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
bash fisco-bcos_amd/tools/gpu_profile_all.sh ${PROF_WLS:-c2} || exit $?
bash fisco-bcos_amd/tools/gpu_bench_check.sh
