"""Diagnosis of concurrent one-launch Merkle roots on two streams (tests/test_gpu_hash.py
test_merkle_one_launch_repeat_two_streams): a width-2 Keccak tree repeated 40 times on one stream while a
partner workload runs on another -- the width-16 one-launch root (merkle_fused_kernel), another width-2
root, or plain torch kernels -- against the root computed alone first.  Every output is allocated and
filled, and the device synchronised, before either stream gets work, so the only interaction is the two
streams' kernels themselves.  Every mode runs on several stream pairs (which streams share a hardware queue,
and so never overlap, depends on creation order); the wall time of both streams against the sum of the two
alone says whether they overlapped.  GPU tool; prints one JSON object.

Round 6: every overlapping pair (both streams in 4.3-5.1 ms against 7.6-8.0 ms serial) gave all 40 roots
right on both streams (profiles/r06_merkle_two_stream_overlap.json).  The test's failures had been the
test's own: it rebound its `tree` variable while the first stream still wrote that tree, and the caching
allocator gave the freed block to the second stream's roots.

usage: merkle_stream_diag.py [PIPES]   (PIPES: host-pointer tx batches run first, each creating a pipeline)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bcos_gpu  # noqa: E402
from bcos_gpu import device  # noqa: E402

REPS = 40


def make_pipes(k):
    """k concurrent host-pointer tx batches: k pipelines (3 streams each) in the library's pool"""
    import threading
    from bcos_gpu import synth, tx
    b = synth.make_batch(0, 600, seed=5)
    pre, po = b.pre.cpu().numpy(), b.pre_off.cpu().numpy().astype(np.uint64)
    sg, so = b.sig.cpu().numpy(), b.sig_off.cpu().numpy().astype(np.uint64)
    th = [threading.Thread(target=tx.verify_packed, args=(bcos_gpu.secp256k1_suite(), pre, po, sg, so))
          for _ in range(k)]
    for t in th:
        t.start()
    for t in th:
        t.join()


def case(rng, n, width):
    leaves = torch.from_numpy(rng.integers(0, 256, size=(n, 32), dtype=np.uint8)).cuda()
    tree = torch.empty((device.merkle_size(n, width), 32), dtype=torch.uint8, device="cuda")
    root = torch.empty(32, dtype=torch.uint8, device="cuda")
    device.merkle_root(device.KECCAK256, width, leaves, tree, root)
    torch.cuda.synchronize()
    return {"leaves": leaves, "tree": tree.clone(), "root": root.clone(), "width": width}


def outputs(c):
    return torch.full_like(c["tree"], 0xAA), torch.full((REPS, 32), 0xAA, dtype=torch.uint8, device="cuda")


def enqueue(c, out, st):
    tree, roots = out
    for r in range(REPS):
        device.merkle_root(device.KECCAK256, c["width"], c["leaves"], tree, roots[r], st)


def bad_reps(c, out):
    return [r for r in range(REPS) if not torch.equal(out[1][r], c["root"])]


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    bcos_gpu.ensure_device(0)
    if len(sys.argv) > 1:
        make_pipes(int(sys.argv[1]))
    rng = np.random.default_rng(78)
    cases = {"w16": case(rng, 100_000, 16), "w2": case(rng, 100_000, 2), "w2_50k": case(rng, 50_000, 2),
             "w2b": case(rng, 100_000, 2)}
    x = torch.randn(4096, 4096, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(8)]
    res = {}
    alone = {}
    for name in ("w16", "w2", "w2_50k", "w2b"):
        o = outputs(cases[name])
        alone[name] = timed(lambda: enqueue(cases[name], o, streams[0]))
    alone["torch"] = timed(lambda: [torch.tanh(x @ x * 1e-3) for _ in range(10)])
    res["alone_ms"] = {k: round(v, 2) for k, v in alone.items()}
    for pair in range(1, 5):
        s0, s1 = streams[0], streams[pair]
        for main_name, partner in (("w2", "w16"), ("w2_50k", "w16"), ("w2", "w2b"), ("w2", "torch")):
            c = cases[main_name]
            mine = outputs(c)
            theirs = outputs(cases[partner]) if partner != "torch" else None
            torch.cuda.synchronize()

            def both():
                if partner == "torch":
                    with torch.cuda.stream(s1):
                        for _ in range(10):
                            torch.tanh(x @ x * 1e-3)
                else:
                    enqueue(cases[partner], theirs, s1)
                enqueue(c, mine, s0)
            ms = timed(both)
            rec = {"ms": round(ms, 2), "serial_ms": round(alone[main_name] + alone[partner], 2),
                   "bad": bad_reps(c, mine)}
            if theirs is not None:
                rec["partner_bad"] = bad_reps(cases[partner], theirs)
            if rec["bad"]:
                b = mine[1][rec["bad"][0]]
                rec["bad_root_fill"] = bool((b == 0xAA).all())
                rec["bad_roots_distinct"] = len({bytes(mine[1][r].cpu().numpy()) for r in rec["bad"]})
            res["pair0_%d %s+%s" % (pair, main_name, partner)] = rec
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
