"""Library A/B of the Merkle root paths: for each path, a child process with the path's environment
switches (read once per process) times bcosgpu_merkle_root on random leaves per (leaves, width) --
mean of back-to-back launches after a warm-up, as bench.py's Merkle legs -- and checks every root
against the first path's.  The parent never touches the GPU.  One JSON line.
  merkle_ab.py [HASHER [NxWIDTH ...]]     HASHER 0 = Keccak256 (default), 1 = SM3
paths: default (the library's choice), sm3_climbx (round 6's SM3 climb kernel with expanded blocks, opt-in),
climb (four-wave one-launch), fused (one-wave one-launch), twolaunch (workgroup + top kernels), nosub (the climb
kernel on the leaves without the subtree kernel first), nosub_lat (nosub on the latency schedule)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PATHS = {"default": {},
         "sm3_climbx": {"BCOSGPU_MERKLE_SM3CLIMB": "1"},
         "climb": {"BCOSGPU_MERKLE_CLIMB": "1"},
         "fused": {"BCOSGPU_MERKLE_CLIMB": "0", "BCOSGPU_MERKLE_FUSED": "1"},
         "twolaunch": {"BCOSGPU_MERKLE_CLIMB": "0", "BCOSGPU_MERKLE_FUSED": "0"},
         "nosub": {"BCOSGPU_MERKLE_NOSUB": "1"},
         "nosub_lat": {"BCOSGPU_MERKLE_NOSUB": "1", "BCOSGPU_MERKLE_LATSCHED": "1"}}

CHILD = r"""
import sys, time, torch
sys.path.insert(0, %r)
import bcos_gpu
from bcos_gpu import device
bcos_gpu.ensure_device(0)
h = int(sys.argv[1])
for spec in sys.argv[2:]:
    n, w = (int(x) for x in spec.split("x"))
    g = torch.Generator(device="cuda"); g.manual_seed(n + w)
    leaves = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    tree = torch.empty((device.merkle_size(n, w), 32), dtype=torch.uint8, device="cuda")
    root = torch.empty(32, dtype=torch.uint8, device="cuda")
    for _ in range(20):
        device.merkle_root(h, w, leaves, tree, root)
    torch.cuda.synchronize()
    reps = 200
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        device.merkle_root(h, w, leaves, tree, root)
    c.record(); c.synchronize()
    print(spec, a.elapsed_time(c) / reps, root.cpu().numpy().tobytes().hex())
""" % os.path.join(ROOT, "fisco-bcos_amd")

args = sys.argv[1:]
hasher = args.pop(0) if args and "x" not in args[0] else "0"
specs = args or ["100000x2", "1000000x2", "100000x16", "1000000x16"]
out, roots = {}, {}
for name, envs in PATHS.items():
    env = dict(os.environ, **envs)
    r = subprocess.run([sys.executable, "-c", CHILD, hasher] + specs, env=env, capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        out[name] = {"error": r.stderr[-400:]}
        break
    res = {}
    for line in r.stdout.splitlines():
        spec, ms, root = line.split()
        res[spec] = round(float(ms), 4)
        if roots.setdefault(spec, root) != root:
            res[spec + "_root_mismatch"] = True
    out[name] = res
    print(name, res, file=sys.stderr, flush=True)
print(json.dumps({"hasher": int(hasher), "merkle_root_ms": out}))
