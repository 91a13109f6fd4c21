# rocprofv3 passes of the bench's Merkle and hash legs (tools/leg_run.py): a kernel trace at steady state
# and separate --pmc passes, summarised per leg into gpurun_out/prof/${R}_pmc_legs.json (tools/leg_prof.py;
# copy into profiles/ so bench.py's Merkle / hash rooflines cite it).
# usage: bash fisco-bcos_amd/tools/gpu_profile_legs.sh [leg names...]
set -o pipefail
R=${R:-r05}
OUT=gpurun_out/prof/legs
mkdir -p $OUT
export TMPDIR=/tmp
RUN="python3 fisco-bcos_amd/tools/leg_run.py"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $RUN 200 "$@" > $OUT/trace.json 2> $OUT/trace.log && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $RUN 5 "$@" > $OUT/fetch.json 2> $OUT/fetch.log && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $RUN 5 "$@" > $OUT/write.json 2> $OUT/write.log && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $RUN 5 "$@" > $OUT/sq.json 2> $OUT/sq.log && \
python3 fisco-bcos_amd/tools/leg_prof.py gpurun_out/prof/${R}_pmc_legs.json --trace $OUT/trace $OUT/trace.json \
  --pmc $OUT/fetch $OUT/fetch.json --pmc $OUT/write $OUT/write.json --pmc $OUT/sq $OUT/sq.json && \
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) gpurun_out/prof/${R}_kernel_stats_legs.csv
rc=$?
echo "profile legs rc=$rc"
exit $rc
