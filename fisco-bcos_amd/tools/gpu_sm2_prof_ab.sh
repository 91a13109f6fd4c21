# rocprofv3 kernel traces of the c2sm2 bench leg under lib_ab/libbcosgpu_A.so (A) and lib/ (B)
mkdir -p gpurun_out
export TMPDIR=/tmp
L=fisco-bcos_amd/lib
cp $L/libbcosgpu.so /tmp/B.so
for v in A B; do
  if [ $v = A ]; then cp fisco-bcos_amd/lib_ab/libbcosgpu_A.so $L/libbcosgpu.so; else cp /tmp/B.so $L/libbcosgpu.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sm2_$v -o run -- python3 bench.py --workload c2sm2 --steps 1000 --warmup 20 --legs "" --no-merkle --no-cpu-baseline --no-extras > gpurun_out/prof_sm2_$v.json 2> gpurun_out/prof_sm2_$v.err || { cp /tmp/B.so $L/libbcosgpu.so; tail -5 gpurun_out/prof_sm2_$v.err; exit 1; }
done
cp /tmp/B.so $L/libbcosgpu.so
for v in A B; do echo "== $v"; find gpurun_out/prof_sm2_$v -name "*kernel_stats.csv" | head -1 | xargs head -6; done
