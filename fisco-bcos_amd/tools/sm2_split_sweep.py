"""Library A/B of the SM2 lane-trio kernel's low-window split (ecc_pair.hip sm2_low_chain): for each
value, a child process with BCOSGPU_SM2_SPLIT set (read once per process) times tx_verify on a 10k-tx
SM2 batch forced onto the trio kernel (median of HIP-event-timed launches after 2 s of warm-up).  The
parent never touches the GPU.  One JSON line.
  sm2_split_sweep.py [SPLIT ...]   (0 = the split-free kernel; any other value = the built-in split)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import sys, time, torch
sys.path.insert(0, %r)
import bcos_gpu
from bcos_gpu import device, synth
bcos_gpu.ensure_device(0)
gpu = bcos_gpu
gpu.set_tx_kernel_policy(1, 0, 2, 1)
n = 10000
b = synth.make_batch(device.SUITE_SM2, n, seed=3)
th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
f = lambda: device.tx_verify(device.SUITE_SM2, b.pre, b.pre_off, b.sig, b.sig_off, th, snd, st)
t0 = time.time()
while time.time() - t0 < 2.0:
    f()
    torch.cuda.synchronize()
ts = []
for _ in range(60):
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); f(); c.record(); c.synchronize()
    ts.append(a.elapsed_time(c))
ts.sort()
print(ts[len(ts) // 2], int((st == 0).sum()))
""" % os.path.join(ROOT, "fisco-bcos_amd")

out = {}
for v in sys.argv[1:] or ["0", "38"]:
    env = dict(os.environ, BCOSGPU_SM2_SPLIT=v)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        out[v] = {"error": r.stderr[-400:]}
        break
    ms, ok = r.stdout.split()[-2:]
    out[v] = {"ms": round(float(ms), 4), "valid": int(ok)}
    print(v, out[v], file=sys.stderr, flush=True)
print(json.dumps({"sm2_trio_split_ms": out}))
