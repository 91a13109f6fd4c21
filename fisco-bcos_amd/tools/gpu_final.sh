# profiles of the remaining workloads, C4 at occupancy 1 (no spills) beside occupancy 2, then the
# default bench line with every profile of this tree in place
mkdir -p gpurun_out
export TMPDIR=/tmp
bash fisco-bcos_amd/tools/gpu_profile_all.sh ${PROF_WLS:-c4 c5 c4comb8} || exit $?
for w in c2 c2sm2 c3 c4 c5 c4comb8; do [ -f gpurun_out/prof/${R:-r03}_pmc_$w.json ] && cp gpurun_out/prof/${R:-r03}_pmc_$w.json profiles/; done
for o in 1 2; do
  BCOSGPU_TXV_OCC=$o timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --warm-seconds 1 --legs= --no-cpu-baseline --no-merkle --no-extras > gpurun_out/bench_c4_occ$o.json 2> gpurun_out/bench_c4_occ$o.err || { tail -20 gpurun_out/bench_c4_occ$o.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_c4_occ$o.json'));print('occ=$o', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
bash fisco-bcos_amd/tools/gpu_bench_check.sh
