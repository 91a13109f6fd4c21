# A/B of the small host-pointer path's staging (BCOSGPU_PIPE_COPY_THREADS) and output (BCOSGPU_PIPE_ZCOUT)
# options on C2's 10k batch (tools/hostpath_probe.py; both read once per process, so one process each),
# interleaved twice.  usage: bash fisco-bcos_amd/tools/small_path_ab.sh  -> gpurun_out/small_ab_<tag>_<k>.json
set -o pipefail
for k in 1 2; do
  for tag in new copy0 zc0 old; do
    case $tag in new) envs="";; copy0) envs="BCOSGPU_PIPE_COPY_THREADS=0";; zc0) envs="BCOSGPU_PIPE_ZCOUT=0";;
      old) envs="BCOSGPU_PIPE_COPY_THREADS=0 BCOSGPU_PIPE_ZCOUT=0";; esac
    env $envs timeout -k 10 120 python3 -u fisco-bcos_amd/tools/hostpath_probe.py 10000 > gpurun_out/small_ab_${tag}_$k.json 2> gpurun_out/small_ab_${tag}_$k.err || { echo "$tag failed"; tail -3 gpurun_out/small_ab_${tag}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/small_ab_${tag}_$k.json'))['secp256k1'][0]
print('$tag $k', {x: round(d[x], 4) for x in ('device_resident_ms', 'verify_packed_ms', 'bare_ctypes_ms', 'pinned_ms') if x in d}, d.get('bare_matches'), d.get('pinned_matches'))"
  done
done
