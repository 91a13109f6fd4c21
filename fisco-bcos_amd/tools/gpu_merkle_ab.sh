# A/B of two libbcosgpu.so builds on the C1 Merkle legs: B = lib/ (the tree), A = lib_ab/libbcosgpu_A.so
mkdir -p gpurun_out
L=fisco-bcos_amd/lib
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash.py -m gpu > gpurun_out/ab_hash.log 2>&1 || { tail -20 gpurun_out/ab_hash.log; exit 1; }
tail -1 gpurun_out/ab_hash.log
cp $L/libbcosgpu.so /tmp/B.so
for i in 1 2 3; do
  for v in B A; do
    if [ $v = A ]; then cp fisco-bcos_amd/lib_ab/libbcosgpu_A.so $L/libbcosgpu.so; else cp /tmp/B.so $L/libbcosgpu.so; fi
    for w in 16 2; do
      echo "$v $(timeout -k 10 60 python3 fisco-bcos_amd/tools/merkle_trace.py 100000 $w 400 | tr '\n' ' ')" || exit 1
    done
  done
done
cp /tmp/B.so $L/libbcosgpu.so
