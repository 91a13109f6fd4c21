# Round 3 re-entry: the -m gpu suite at the current tree, the default bench line, then rocprofv3
# trace + PMC passes of the headline workloads (C2, C2-SM2) under this tree's kernel sources.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_default.err; [ $rc -eq 0 ] || exit $rc
bash fisco-bcos_amd/tools/gpu_profile_all.sh ${PROF_WLS:-c2 c2sm2}
