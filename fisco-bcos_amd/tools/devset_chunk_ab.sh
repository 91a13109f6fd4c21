# Device-set legs (tools/devset_probe.py, {0,0}) at forced pipeline chunk sizes (BCOSGPU_PIPE_CHUNK, which
# also drops the head chunk) against the default, alternated twice.  -> gpurun_out/dsc_<tag>_<k>.json
#   usage: bash fisco-bcos_amd/tools/devset_chunk_ab.sh [TAGS...]   (default | c<chunk>; default: all four)
set -o pipefail
TAGS=${@:-default c65536 c98304 c196608}
for k in 1 2; do
  for tag in $TAGS; do
    case $tag in default) envs="BCOSGPU_X=1";; c*) envs="BCOSGPU_PIPE_CHUNK=${tag#c}";; esac
    env $envs timeout -k 10 150 python3 -u fisco-bcos_amd/tools/devset_probe.py 0,0 2 > gpurun_out/dsc_${tag}_$k.json 2> gpurun_out/dsc_${tag}_$k.err || { echo "$tag failed"; tail -3 gpurun_out/dsc_${tag}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/dsc_${tag}_$k.json'))
print('$tag $k', {w: (round(v['tx_s']/1e6,2), v['matches_single_device']) for w, v in d.items() if isinstance(v, dict) and 'tx_s' in v})"
  done
done
