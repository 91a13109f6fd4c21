# rocprofv3 kernel-trace + PMC passes for every bench workload at the current tree, summarised into
# gpurun_out/prof/r02_pmc_<wl>.json (copy into profiles/ to make bench.py's traffic cite them).
# usage: bash fisco-bcos_amd/tools/gpu_profile_all.sh [workloads...]
set -o pipefail
mkdir -p gpurun_out/prof
WLS=${@:-c2 c2sm2 c3 c4 c5}
for wl in $WLS; do
  case $wl in c2|c2sm2) st=30;; *) st=3;; esac
  bash fisco-bcos_amd/tools/gpu_profile.sh $wl $st 240 || exit $?
  python3 fisco-bcos_amd/tools/prof_summary.py gpurun_out/prof/r02_pmc_$wl.json gpurun_out/prof/$wl/trace \
    gpurun_out/prof/$wl/fetch gpurun_out/prof/$wl/write gpurun_out/prof/$wl/sq gpurun_out/prof/$wl/valu || exit $?
  cp $(find gpurun_out/prof/$wl/trace -name '*kernel_stats.csv' | head -1) gpurun_out/prof/r02_kernel_stats_$wl.csv
done
echo done
