# Round 3 profile refresh, part 1: rocprofv3 trace + PMC passes of C2, C2-SM2, C3 under the current
# kernel sources, then the default bench line with those profiles in place.
mkdir -p gpurun_out
export TMPDIR=/tmp
bash fisco-bcos_amd/tools/gpu_profile_all.sh c2 c2sm2 c3 || exit $?
for w in c2 c2sm2 c3; do cp gpurun_out/prof/r03_pmc_$w.json profiles/; done
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_default.err; exit $rc
