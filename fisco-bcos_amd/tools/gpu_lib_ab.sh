# A/B of two libbcosgpu.so builds on one bench workload: B = lib/ (the tree), A = lib_ab/libbcosgpu_A.so.
# usage: bash fisco-bcos_amd/tools/gpu_lib_ab.sh <workload> [steps]
mkdir -p gpurun_out
L=fisco-bcos_amd/lib
WL=${1:-c2sm2}; ST=${2:-2000}
cp $L/libbcosgpu.so /tmp/B.so
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then cp fisco-bcos_amd/lib_ab/libbcosgpu_A.so $L/libbcosgpu.so; else cp /tmp/B.so $L/libbcosgpu.so; fi
    timeout -k 10 120 python3 bench.py --workload $WL --steps $ST --warmup 20 --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { cp /tmp/B.so $L/libbcosgpu.so; tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4))"
  done
done
cp /tmp/B.so $L/libbcosgpu.so
