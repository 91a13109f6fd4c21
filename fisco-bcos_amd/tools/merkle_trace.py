"""Merkle C1 (merkleBench: width-16 root over 100k leaves) in a loop, for rocprofv3 --kernel-trace:
per-level kernel durations and the gaps between dependent launches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))

import numpy as np
import torch

import bcos_gpu
from bcos_gpu import device

bcos_gpu.ensure_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
width = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
leaves = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=(n, 32), dtype=np.uint8)).cuda()
for h in (device.KECCAK256, device.SM3):
    tree = torch.empty((device.merkle_size(n, width), 32), dtype=torch.uint8, device="cuda")
    root = torch.empty(32, dtype=torch.uint8, device="cuda")
    for _ in range(5):
        device.merkle_root(h, width, leaves, tree, root)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        device.merkle_root(h, width, leaves, tree, root)
    torch.cuda.synchronize()
    print("hasher", h, "ms", (time.perf_counter() - t0) / reps * 1e3, "width", width)
