# rocprofv3 passes for one bench workload on the MI355X box: kernel trace + stats, then separate
# --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a pass), each under its own time limit.
# usage: bash fisco-bcos_amd/tools/gpu_profile.sh <workload> <steps> <limit_s> [tag]
# writes gpurun_out/prof/<tag>/{trace,fetch,write,sq,valu}/ (tag defaults to the workload; the caller's
# environment, e.g. BCOSGPU_TABLES=small, applies to every pass)
set -o pipefail
WL=${1:-c2}; STEPS=${2:-10}; LIM=${3:-180}; TAG=${4:-$WL}
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --workload $WL --steps $STEPS --warmup 2 --warm-seconds 0 --legs= --no-cpu-baseline --no-merkle --no-extras --no-hashes --devset none --detail-out="
# the trace pass at steady state: >= 2 s of warm-up launches and >= 2 s of timed ones, so the kernel's
# average duration is the clock-settled one the bench line reports (the PMC passes serialise dispatches
# and only count, so they stay short)
BT="python3 bench.py --workload $WL --steps $((STEPS * 100)) --warmup 2 --warm-seconds 2 --legs= --no-cpu-baseline --no-merkle --no-extras --no-hashes --devset none --detail-out="
timeout -k 10 $LIM rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BT > $OUT/trace.log 2>&1 && \
timeout -s KILL $LIM rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 && \
timeout -s KILL $LIM rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 && \
timeout -s KILL $LIM rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 && \
timeout -s KILL $LIM rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/valu -o run -- $B > $OUT/valu.log 2>&1
rc=$?
echo "profile $TAG rc=$rc"
exit $rc
