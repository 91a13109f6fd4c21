# Device-set legs on {0,0} (tools/devset_probe.py): partial chunk first for shards sharing a device (the
# default) against last (BCOSGPU_PIPE_REMFIRST=0), alternated three times.
set -o pipefail
for k in 1 2 3; do
  for tag in default rem0; do
    case $tag in default) envs="BCOSGPU_X=1";; rem0) envs="BCOSGPU_PIPE_REMFIRST=0";; esac
    env $envs timeout -k 10 150 python3 -u fisco-bcos_amd/tools/devset_probe.py 0,0 2 > gpurun_out/dsr_${tag}_$k.json 2> gpurun_out/dsr_${tag}_$k.err || { echo "$tag failed"; tail -3 gpurun_out/dsr_${tag}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/dsr_${tag}_$k.json'))
print('$tag $k', {w: (round(v['tx_s']/1e6,2), v['matches_single_device']) for w, v in d.items() if isinstance(v, dict) and 'tx_s' in v})"
  done
done
