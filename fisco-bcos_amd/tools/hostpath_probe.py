"""Where a host-pointer batch call's time goes (bcosgpu_tx_verify_batch): the device-resident kernel alone,
the Python wrapper (tx.verify_packed: output allocation + ctypes), the bare ctypes call into preallocated
numpy outputs, and the same with pinned host inputs and outputs.  Medians over `reps` calls, per batch size.
GPU tool (not a test); prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bcos_gpu  # noqa: E402
from bcos_gpu import device, synth, tx  # noqa: E402
from bcos_gpu._lib import check, lib  # noqa: E402
from bcos_gpu.crypto import _ptr  # noqa: E402


def med(f, reps):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def probe(suite, n, reps):
    b = synth.make_batch(suite, n, seed=0xC2)
    th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")

    def dev():
        device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, th, snd, st)
        torch.cuda.synchronize()
    out = {"n": n, "device_resident_ms": med(dev, reps)}
    pre = np.ascontiguousarray(b.pre.cpu().numpy())
    po = np.ascontiguousarray(b.pre_off.cpu().numpy().astype(np.uint64))
    sg = np.ascontiguousarray(b.sig.cpu().numpy())
    so = np.ascontiguousarray(b.sig_off.cpu().numpy().astype(np.uint64))
    s = bcos_gpu.sm_suite() if suite else bcos_gpu.secp256k1_suite()
    want = tx.verify_packed(s, pre, po, sg, so)
    out["verify_packed_ms"] = med(lambda: tx.verify_packed(s, pre, po, sg, so), reps)
    h, sd, stt = (np.zeros_like(x) for x in want)

    def bare(pre=pre, po=po, sg=sg, so=so, h=h, sd=sd, stt=stt):
        check(lib().bcosgpu_tx_verify_batch(suite, _ptr(pre), _ptr(po), _ptr(sg), _ptr(so), n, _ptr(h), _ptr(sd),
                                            _ptr(stt)))
    out["bare_ctypes_ms"] = med(bare, reps)
    out["bare_matches"] = all(np.array_equal(x, y) for x, y in zip((h, sd, stt), want))
    pin = [torch.from_numpy(x).pin_memory().numpy() for x in (pre, po, sg, so)]
    pout = [torch.from_numpy(np.zeros_like(x)).pin_memory().numpy() for x in want]
    out["pinned_ms"] = med(lambda: bare(*pin, *pout), reps)
    out["pinned_matches"] = all(np.array_equal(x, y) for x, y in zip(pout, want))
    if n <= 65536:  # A/B of the small-batch pipeline choices (txpipe.hip test hooks)
        for name, env in (("staged", {}), ("pageable", {"BCOSGPU_PIPE_STAGED": "0"}),
                          ("halves_pageable", {"BCOSGPU_PIPE_CHUNK": str((n + 1) // 2)})):
            old = {k: os.environ.get(k) for k in ("BCOSGPU_PIPE_CHUNK", "BCOSGPU_PIPE_STAGED")}
            for k in old:
                os.environ.pop(k, None)
            os.environ.update(env)
            out["bare_" + name + "_ms"] = med(bare, reps)
            for k, v in old.items():
                os.environ.pop(k, None)
                if v is not None:
                    os.environ[k] = v
        half = n // 2
        thh, sdh, sth = th[:half], snd[:half], st[:half]

        def dev_half():
            device.tx_verify(suite, b.pre, b.pre_off[: half + 1], b.sig, b.sig_off[: half + 1], thh, sdh, sth)
            torch.cuda.synchronize()
        out["device_resident_half_ms"] = med(dev_half, reps)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        th2, sd2, st2 = th[half:], snd[half:], st[half:]
        po2, so2 = b.pre_off[half:], b.sig_off[half:]

        def dev_two():
            device.tx_verify(suite, b.pre, b.pre_off[: half + 1], b.sig, b.sig_off[: half + 1], thh, sdh, sth,
                             stream=s1)
            device.tx_verify(suite, b.pre, po2, b.sig, so2, th2, sd2, st2, stream=s2)
            torch.cuda.synchronize()
        out["device_two_halves_concurrent_ms"] = med(dev_two, reps)
    mb = (pre.nbytes + po.nbytes + sg.nbytes + so.nbytes) / 1e6
    out["h2d_MB"], out["d2h_MB"] = round(mb, 3), round(sum(x.nbytes for x in want) / 1e6, 3)
    return out


def main():
    bcos_gpu.ensure_device(0)
    sizes = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["10000", "131072", "1000000"])]
    res = {"secp256k1": [probe(0, n, 50 if n <= 20000 else 5) for n in sizes]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
