"""The bench's Merkle and hash legs (bench.MERKLE_SPECS, bench.HASH_SPECS) on the library's default paths,
for rocprofv3:
  rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 fisco-bcos_amd/tools/leg_run.py [REPS] [NAME ...]
  rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d DIR -o run -- python3 .../leg_run.py 5

Per leg: inputs built (torch kernels), a separator fill, REPS roots / batches back to back, a separator
fill.  tools/leg_prof.py assigns the library dispatches between a leg's two separators to it (the legs run
in the printed order).  Prints one JSON line {"order": [...], "ms": {leg: ms per root / batch}}."""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import bcos_gpu  # noqa: E402
import bench  # noqa: E402
from bcos_gpu import device  # noqa: E402


def main():
    args = sys.argv[1:]
    reps = int(args.pop(0)) if args and args[0].isdigit() else 200
    bcos_gpu.ensure_device(0)
    specs = [("merkle", bench.merkle_name(n, h, w), (n, h, w)) for n, h, w in bench.MERKLE_SPECS]
    specs += [("hash", name, (h, n, ln)) for name, h, n, ln in bench.HASH_SPECS]
    if args:
        specs = [s for s in specs if s[1] in args]
    sep = torch.empty(7, dtype=torch.int32, device="cuda")  # (torch.zeros would launch a fill of its own)
    order, ms = [], {}
    for kind, name, spec in specs:
        if kind == "merkle":
            n, h, w = spec
            leaves = bench.merkle_inputs(n)
            tree = torch.empty((device.merkle_size(n, w), 32), dtype=torch.uint8, device="cuda")
            root = torch.empty(32, dtype=torch.uint8, device="cuda")
            hasher = bench._hasher(h)

            def fn():
                device.merkle_root(hasher, w, leaves, tree, root)
            bufs = (leaves, tree, root)
        else:
            h, n, ln = spec
            data, off = bench.hash_inputs(n, ln)
            dig = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
            hasher = bench._hasher(h)

            def fn():
                device.hash_batch(hasher, data, off, dig)
            bufs = (data, off, dig)
        for _ in range(min(reps, 20)):  # warm-up (before the leg's first separator)
            fn()
        torch.cuda.synchronize()
        sep.fill_(1)
        a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        c.record()
        sep.fill_(2)
        torch.cuda.synchronize()
        ms[name] = round(a.elapsed_time(c) / reps, 5)
        order.append(name)
        print(name, ms[name], file=sys.stderr, flush=True)
        del bufs, fn
        torch.cuda.empty_cache()
    print(json.dumps({"reps": reps, "order": order, "ms": ms}))


if __name__ == "__main__":
    main()
