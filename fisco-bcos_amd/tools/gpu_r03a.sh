# Round 3, first GPU call: the full -m gpu suite (new: SigIO kernel paths, coalesced single calls,
# 64-thread adapter test), the occupancy sweep for the one-lane kernel's rounds x latency rule, and a
# short bench (C2 + the interface legs).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -80; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u fisco-bcos_amd/tools/small_sweep.py 65536,98304,125952,131072,196608,262144,524288 > gpurun_out/occ_sweep.json 2> gpurun_out/occ_sweep.log
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/occ_sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --legs "" --no-merkle --no-cpu-baseline > gpurun_out/bench_a.json 2> gpurun_out/bench_a.log
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_a.json; exit $rc
