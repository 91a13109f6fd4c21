# One GPU call: the -m gpu suite (full-size parity included), then the rocprofv3 counter list.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -70; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
exit 0
