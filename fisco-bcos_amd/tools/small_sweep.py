"""Kernel time of every small-batch variant against the batch size (the data behind the automatic
choice in ecc_txv.hip): secp256k1 and SM2, row (secp256k1) / lane-trio / wave-pair / one-lane at occupancy 1 and 2, each
forced with bcosgpu_set_tx_kernel_policy, and the automatic policy; median of HIP-event-timed launches
after a warm-up.  One JSON line.
  small_sweep.py [SIZES]          Transaction::verify batches (bcosgpu_tx_verify_batch_dev)
  small_sweep.py verify [SIZES]   known-key verify batches (bcosgpu_verify_batch_dev): secp256k1 trio /
                                  one-lane, SM2 trio / pair / one-lane occupancy 1 and 2, and auto"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))

import torch

import bcos_gpu
from bcos_gpu import device, synth

bcos_gpu.ensure_device(0)
VARIANTS = {"trio": (1, 0, 2, 1), "row": (1, 0, 3, 1), "pair": (1, 0, 1, 1), "occ1": (0, 1, 0, 1),
            "occ2": (0, 2, 0, 1), "auto": (-1, 0, 2, 1)}  # row: ecc_row.hip (secp256k1 recovery, SM2 verify)
args = sys.argv[1:]
mode = args.pop(0) if args and args[0] == "verify" else "tx"
# sizes: one comma-separated argument or several arguments (tools/gpu_run.sh turns commas into spaces)
sizes = [int(x) for x in (",".join(args) if args else "10240,12800,16384,20480,24576,32768").split(",") if x]
out = {}


def median_ms(fn, warm=20, reps=40):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return round(ts[len(ts) // 2], 4)


if mode == "verify":
    from bcos_gpu import _lib
    L = _lib.lib()
    m = max(sizes)
    for suite in (0, 1):
        g = torch.Generator(device="cuda")
        g.manual_seed(11 + suite)
        sk = torch.randint(0, 256, (m, 32), dtype=torch.uint8, device="cuda", generator=g)
        sk[:, 0] &= 0x7F
        sk[:, 31] |= 1
        h = torch.randint(0, 256, (m, 32), dtype=torch.uint8, device="cuda", generator=g)
        ok = torch.empty(m, dtype=torch.uint8, device="cuda")
        if suite == 0:
            pub = torch.empty((m, 64), dtype=torch.uint8, device="cuda")
            sig = torch.empty((m, 65), dtype=torch.uint8, device="cuda")
            device.secp256k1_sign(sk, h, pub, sig, ok)
            variants = {"trio": (1, 0, 2, 1), "row": (1, 0, 3, 1), "onelane": (0, 0, 2, 1), "auto": (-1, 0, 2, 1)}
        else:
            sig = torch.empty((m, 128), dtype=torch.uint8, device="cuda")
            device.sm2_sign(sk, h, sig, ok)
            pub = sig[:, 64:].contiguous()
            variants = {"trio": (1, 0, 2, 1), "pair": (1, 0, 1, 1), "occ1": (0, 1, 0, 1), "occ2": (0, 2, 0, 1),
                        "auto": (-1, 0, 2, 1)}
        for n in sizes:
            for name, pol in variants.items():
                bcos_gpu.set_tx_kernel_policy(*pol)
                out["%s_%d_%s" % ("secp" if suite == 0 else "sm2", n, name)] = median_ms(
                    lambda: _lib.check(L.bcosgpu_verify_batch_dev(suite, pub.data_ptr(), h.data_ptr(), sig.data_ptr(),
                                                                  sig.shape[1], n, ok.data_ptr(), None)))
                torch.cuda.synchronize()
                assert bool(ok[:n].all()), (suite, n, name)
            print(n, {k: v for k, v in out.items() if ("_%d_" % n) in k}, file=sys.stderr, flush=True)
    bcos_gpu.set_tx_kernel_policy()
    print(json.dumps(out))
    sys.exit(0)

for suite in (0, 1):
    big = synth.make_batch(suite, max(sizes), seed=3 + suite)
    for n in sizes:
        po = big.pre_off[: n + 1]
        so = big.sig_off[: n + 1]
        th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        for name, pol in VARIANTS.items():
            bcos_gpu.set_tx_kernel_policy(*pol)
            for _ in range(30):
                device.tx_verify(suite, big.pre, po, big.sig, so, th, snd, st)
            ts = []
            for _ in range(60):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                device.tx_verify(suite, big.pre, po, big.sig, so, th, snd, st)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            ts.sort()
            out["%s_%d_%s" % ("secp" if suite == 0 else "sm2", n, name)] = round(ts[len(ts) // 2], 4)
        print(n, {k: v for k, v in out.items() if ("_%d_" % n) in k}, file=sys.stderr, flush=True)
bcos_gpu.set_tx_kernel_policy()
print(json.dumps(out))
