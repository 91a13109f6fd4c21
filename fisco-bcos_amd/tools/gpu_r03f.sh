# Round 3 profile refresh, part 2: C4, C5 and C4 on the 8-bit comb tables.
mkdir -p gpurun_out
export TMPDIR=/tmp
bash fisco-bcos_amd/tools/gpu_profile_all.sh c4 c5 c4comb8
