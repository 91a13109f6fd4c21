# rocprofv3 kernel-trace + PMC passes for every bench workload at the current tree, summarised into
# gpurun_out/prof/<round>_pmc_<wl>.json (copy into profiles/ to make bench.py's traffic cite them).
# usage: bash fisco-bcos_amd/tools/gpu_profile_all.sh [workloads...]
set -o pipefail
mkdir -p gpurun_out/prof
# (tag c4comb8: the C4 workload on the 8-bit comb tables, BCOSGPU_TABLES=small, to split the traffic)
WLS=${@:-c2 c2sm2 c3 c4 c5 c4comb8}
for tag in $WLS; do
  wl=$tag; envs=""
  [ $tag = c4comb8 ] && { wl=c4; envs="BCOSGPU_TABLES=small"; }
  case $wl in c2|c2sm2) st=30;; *) st=3;; esac
  env $envs bash fisco-bcos_amd/tools/gpu_profile.sh $wl $st 240 $tag || exit $?
  python3 fisco-bcos_amd/tools/prof_summary.py gpurun_out/prof/${R:-r05}_pmc_$tag.json gpurun_out/prof/$tag/trace \
    gpurun_out/prof/$tag/fetch gpurun_out/prof/$tag/write gpurun_out/prof/$tag/sq gpurun_out/prof/$tag/valu || exit $?
  cp $(find gpurun_out/prof/$tag/trace -name '*kernel_stats.csv' | head -1) gpurun_out/prof/${R:-r05}_kernel_stats_$tag.csv
done
echo done
