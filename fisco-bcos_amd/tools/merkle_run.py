"""Merkle roots on the library's default paths, for a kernel trace:
  rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 fisco-bcos_amd/tools/merkle_run.py HxNxW ...
H = 0 (Keccak256) / 1 (SM3), N leaves, width W.  Per spec: 20 warm-up roots, then 200 back-to-back roots
timed with events (as bench.py's Merkle legs); prints one JSON line {spec: ms per root}."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bcos_gpu  # noqa: E402
from bcos_gpu import device  # noqa: E402

bcos_gpu.ensure_device(0)
out = {}
for spec in sys.argv[1:] or ["0x100000x16", "1x100000x16", "0x100000x2", "1x100000x2"]:
    h, n, w = (int(x) for x in spec.split("x"))
    g = torch.Generator(device="cuda")
    g.manual_seed(n + w)
    leaves = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    tree = torch.empty((device.merkle_size(n, w), 32), dtype=torch.uint8, device="cuda")
    root = torch.empty(32, dtype=torch.uint8, device="cuda")
    for _ in range(20):
        device.merkle_root(h, w, leaves, tree, root)
    torch.cuda.synchronize()
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        device.merkle_root(h, w, leaves, tree, root)
    c.record()
    c.synchronize()
    out[spec] = round(a.elapsed_time(c) / 200, 4)
    print(spec, out[spec], file=sys.stderr, flush=True)
    del leaves, tree
    torch.cuda.empty_cache()
print(json.dumps({"merkle_root_ms": out}))
