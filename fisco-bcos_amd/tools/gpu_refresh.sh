# profiles + default bench at the current tree (one gpurun call)
bash fisco-bcos_amd/tools/gpu_profile_all.sh && bash fisco-bcos_amd/tools/gpu_bench_check.sh
