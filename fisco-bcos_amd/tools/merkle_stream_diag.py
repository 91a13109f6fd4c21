"""Diagnosis of concurrent one-launch Merkle roots on two streams (tests/test_gpu_hash.py
test_merkle_one_launch_repeat_two_streams): width 16 (merkle_fused_kernel) on one stream and width 2
(merkle_climb_kernel) on another, 40 roots each, against each tree computed alone first; reports which
repetitions differ and at which tree level.  GPU tool; prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bcos_gpu  # noqa: E402
from bcos_gpu import device  # noqa: E402


def levels(n, w):
    out, pos, m = [], 0, n
    while m > 1:
        m = (m + w - 1) // w
        out.append((pos, m))
        pos += m + 1
    return out


def main():
    bcos_gpu.ensure_device(0)
    rng = np.random.default_rng(78)
    n, reps = 100_000, 40
    cases = []
    for width in (16, 2):
        leaves = torch.from_numpy(rng.integers(0, 256, size=(n, 32), dtype=np.uint8)).cuda()
        tree = torch.empty((device.merkle_size(n, width), 32), dtype=torch.uint8, device="cuda")
        root = torch.empty(32, dtype=torch.uint8, device="cuda")
        device.merkle_root(device.KECCAK256, width, leaves, tree, root)
        torch.cuda.synchronize()
        cases.append((width, leaves, tree.clone(), root.clone()))
    out = {}
    for mode in ("alone_w2", "concurrent", "concurrent_trees"):
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        res = []
        for k, st in enumerate(streams):
            width, leaves, want_tree, want_root = cases[k]
            if mode == "alone_w2" and width != 2:
                res.append(None)
                continue
            trees = [torch.empty_like(want_tree) for _ in range(reps if mode == "concurrent_trees" else 1)]
            roots = torch.zeros((reps, 32), dtype=torch.uint8, device="cuda")
            with torch.cuda.stream(st):
                for r in range(reps):
                    device.merkle_root(device.KECCAK256, width, leaves, trees[r % len(trees)], roots[r], st)
            res.append((width, trees, roots, want_tree, want_root))
        torch.cuda.synchronize()
        rec = {}
        for item in res:
            if item is None:
                continue
            width, trees, roots, want_tree, want_root = item
            bad = [r for r in range(reps) if not torch.equal(roots[r], want_root)]
            d = {"bad_reps": bad}
            if mode == "concurrent_trees":
                lv = levels(n, width)
                first_bad_level = {}
                for r in range(reps):
                    diff = (trees[r] != want_tree).any(dim=1).nonzero().flatten().tolist()
                    if diff:
                        e = diff[0]
                        lvl = max(i for i, (p, _) in enumerate(lv) if p <= e)
                        first_bad_level[r] = {"entry": e, "level": lvl, "entries_bad": len(diff)}
                d["first_bad"] = first_bad_level
            rec["w%d" % width] = d
        out[mode] = rec
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
