set -o pipefail
for k in 1 2; do
  for d in 128 0; do
    BCOSGPU_COALESCE_DEEP=$d timeout -k 10 300 python -u fisco-bcos_amd/tools/callbench_sweep.py gpurun_out 64,128,256 4,8 4 > gpurun_out/lfd_${d}_$k.jsonl 2>/dev/null || exit 1
    python3 -c "
import json
for l in open('gpurun_out/lfd_${d}_$k.jsonl'):
    r=json.loads(l); c=r['coalescer']; h=r['host']
    print('deep=$d k=$k', r['suite'], r['threads'], r['slots'], int(r['calls_per_s']), r['latency_us']['p50'], r['latency_us']['p99'], r['mismatches'], c['calls_per_batch'], h['cores_busy'])"
  done
done
