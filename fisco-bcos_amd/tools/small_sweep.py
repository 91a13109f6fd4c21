"""Kernel time of every small-batch variant against the batch size (the data behind the automatic
choice in ecc_txv.hip): secp256k1 and SM2, lane-trio / wave-pair / one-lane at occupancy 1 and 2, each
forced with bcosgpu_set_tx_kernel_policy, and the automatic policy; median of HIP-event-timed launches
after a warm-up.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))

import torch

import bcos_gpu
from bcos_gpu import device, synth

bcos_gpu.ensure_device(0)
VARIANTS = {"trio": (1, 0, 2, 1), "pair": (1, 0, 1, 1), "occ1": (0, 1, 0, 1), "occ2": (0, 2, 0, 1),
            "auto": (-1, 0, 2, 1)}
sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "10240,12800,16384,20480,24576,32768").split(",")]
out = {}
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
