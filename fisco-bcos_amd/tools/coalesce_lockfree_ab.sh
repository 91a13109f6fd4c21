# Same-box A/B of the coalescer's lock-free arrivals (BCOSGPU_COALESCE_LOCKFREE=1, default, against 0):
# callbench at 16 / 64 / 256 threads, 4 slots, alternated twice.  -> gpurun_out/lf_<v>_<k>.jsonl
set -o pipefail
for k in 1 2; do
  for v in 1 0; do
    BCOSGPU_COALESCE_LOCKFREE=$v timeout -k 10 300 python -u fisco-bcos_amd/tools/callbench_sweep.py gpurun_out 16,64,256 4 4 > gpurun_out/lf_${v}_$k.jsonl 2>/dev/null || exit 1
    python3 -c "
import json
for l in open('gpurun_out/lf_${v}_$k.jsonl'):
    r=json.loads(l); c=r['coalescer']; h=r['host']
    print('lockfree=$v k=$k', r['suite'], r['threads'], int(r['calls_per_s']), r['latency_us']['p50'], r['latency_us']['p99'], r['mismatches'], r['engine_errors'], c['lock_us_per_call'], h['cores_busy'], h['cpu_us_per_call'])"
  done
done
