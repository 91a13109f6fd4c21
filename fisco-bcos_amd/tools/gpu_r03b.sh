# Coalescer sweep (threads x slots) + a kernel/copy trace of the 64-thread single-call run.
mkdir -p gpurun_out/cb
export TMPDIR=/tmp
timeout -k 10 600 python3 -u fisco-bcos_amd/tools/callbench_sweep.py gpurun_out/cb > gpurun_out/cb/sweep.jsonl 2> gpurun_out/cb/sweep.log
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/cb/sweep.jsonl; tail -5 gpurun_out/cb/sweep.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cb/prof -o cb --output-format csv -- $GRAFT_REPO_ROOT/fisco-bcos_amd/lib/callbench $GRAFT_REPO_ROOT/gpurun_out/cb/callbench_0.bin 64 500 > $GRAFT_REPO_ROOT/gpurun_out/cb/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/cb/prof.log; rm -f $GRAFT_REPO_ROOT/gpurun_out/cb/*.bin; exit $rc
