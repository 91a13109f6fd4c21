set -o pipefail
for k in 1 2 3; do
  for d in 128 0; do
    BCOSGPU_COALESCE_DEEP=$d timeout -k 10 200 python -u fisco-bcos_amd/tools/callbench_sweep.py gpurun_out 256 4 4 > gpurun_out/deep_${d}_$k.jsonl 2>/dev/null || exit 1
    python3 -c "
import json
for l in open('gpurun_out/deep_${d}_$k.jsonl'):
    r=json.loads(l); c=r['coalescer']; h=r['host']
    print('deep=$d k=$k', r['suite'], int(r['calls_per_s']), r['latency_us']['p50'], r['latency_us']['p99'], c['calls_per_batch'], h['cores_busy'], h['cpu_us_per_call'])"
  done
done
