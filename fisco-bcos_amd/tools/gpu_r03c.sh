# Round 3: the lane-pair Keccak check, the -m gpu suite at the current tree, the default bench line,
# a Merkle C1 A/B (lane-pair levels off / on), then rocprofv3 trace + PMC passes of the headline
# workloads (C2, C2-SM2) under this tree's kernel sources.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 fisco-bcos_amd/lib/keccakpair_check > gpurun_out/keccakpair.json 2>&1
rc=$?; echo "keccakpair rc=$rc"; cat gpurun_out/keccakpair.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do for w in 16 2; do
  echo "pair=$v w=$w $(BCOSGPU_MERKLE_PAIR=$v timeout -k 10 60 python3 fisco-bcos_amd/tools/merkle_trace.py 100000 $w 400 | tr '\n' ' ')" || exit 1
done; done; done 2>&1 | tee gpurun_out/merkle_ab.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_default.err; [ $rc -eq 0 ] || exit $rc
bash fisco-bcos_amd/tools/gpu_profile_all.sh ${PROF_WLS:-c2 c2sm2}
