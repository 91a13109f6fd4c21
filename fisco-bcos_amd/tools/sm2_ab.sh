# A/B of SM2 trio-kernel variants on c2sm2 (10k SM2 txs): the default library, libraries rebuilt with more
# unrolled doublings per window (tools/build_ab.sh sm2unroll2 / sm2unroll4 ecc_pair -DkSm2DblUnroll=N) and
# the round-3 schedule without the low-window chains (BCOSGPU_SM2_SPLIT=0), alternated twice.
#   -> gpurun_out/sm2ab_<tag>_<k>.json (bench lines)
set -o pipefail
A="--workload c2sm2 --steps 3000 --warmup 20 --legs= --no-cpu-baseline --no-merkle --no-extras --no-hashes --devset none --detail-out="
cp fisco-bcos_amd/lib/libbcosgpu.so /tmp/libbcosgpu.main.so
for k in 1 2; do
  for tag in default unroll2 unroll4 split0; do
    envs="BCOSGPU_X=1"
    case $tag in unroll*) cp fisco-bcos_amd/lib_ab/sm2$tag/libbcosgpu.so fisco-bcos_amd/lib/;; split0) envs="BCOSGPU_SM2_SPLIT=0";; esac
    env $envs timeout -k 10 200 python3 -u bench.py $A > gpurun_out/sm2ab_${tag}_$k.json 2> gpurun_out/sm2ab_${tag}_$k.err
    rc=$?
    cp /tmp/libbcosgpu.main.so fisco-bcos_amd/lib/libbcosgpu.so
    [ $rc -eq 0 ] || { echo "$tag failed"; tail -3 gpurun_out/sm2ab_${tag}_$k.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/sm2ab_${tag}_$k.json').read().strip().splitlines()[-1])
print('$tag $k', round(l['ms_per_step'], 4), l['roofline'].get('kernel_ms'))"
  done
done
