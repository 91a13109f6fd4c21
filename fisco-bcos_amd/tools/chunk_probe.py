"""Chunking cost of the tx pipeline at 1M secp256k1 txs (txpipe.hip): the device-resident single launch, the
same batch as device-resident chunk launches on one / two alternating streams, and the host-pointer call
(bcosgpu_tx_verify_batch) at several chunk sizes and stream counts (test hooks BCOSGPU_PIPE_CHUNK /
BCOSGPU_PIPE_STREAMS).  Medians in ms.  GPU tool; prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bcos_gpu  # noqa: E402
from bcos_gpu import device, synth  # noqa: E402
from bcos_gpu._lib import check, lib  # noqa: E402
from bcos_gpu.crypto import _ptr  # noqa: E402
from hostpath_probe import med  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1_000_000
    reps = 5
    bcos_gpu.ensure_device(0)
    b = synth.make_batch(0, n, seed=0xC4)
    th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    sd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {"n": n}

    def resident(chunk=None, nstreams=1):
        ss = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]

        def f():
            c = chunk or n
            for k, a in enumerate(range(0, n, c)):
                e = min(n, a + c)
                device.tx_verify(0, b.pre, b.pre_off[a:e + 1], b.sig, b.sig_off[a:e + 1], th[a:e], sd[a:e], st[a:e],
                                 stream=ss[k % nstreams])
            torch.cuda.synchronize()
        return f
    out["resident_single"] = med(resident(), reps)
    for c in (131072, 262144, 524288):
        for ns in (1, 2):
            out["resident_chunk%d_s%d" % (c, ns)] = med(resident(c, ns), reps)
    pre = np.ascontiguousarray(b.pre.cpu().numpy())
    po = np.ascontiguousarray(b.pre_off.cpu().numpy().astype(np.uint64))
    sg = np.ascontiguousarray(b.sig.cpu().numpy())
    so = np.ascontiguousarray(b.sig_off.cpu().numpy().astype(np.uint64))
    h, s2, t2 = np.zeros((n, 32), np.uint8), np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)

    def bare():
        check(lib().bcosgpu_tx_verify_batch(0, _ptr(pre), _ptr(po), _ptr(sg), _ptr(so), n, _ptr(h), _ptr(s2), _ptr(t2)))
    if "--quick" not in sys.argv:
        for c in (131072, 262144, 524288):
            for ns in ("1", "2"):
                os.environ["BCOSGPU_PIPE_CHUNK"], os.environ["BCOSGPU_PIPE_STREAMS"] = str(c), ns
                out["host_chunk%d_s%s" % (c, ns)] = med(bare, reps)
        os.environ.pop("BCOSGPU_PIPE_CHUNK")
        os.environ.pop("BCOSGPU_PIPE_STREAMS")
    for rep in range(2):  # alternated A/B of the head chunk and of the partial chunk first
        os.environ["BCOSGPU_PIPE_HEAD"] = "0"
        out["host_no_head_%d" % rep] = med(bare, reps)
        os.environ["BCOSGPU_PIPE_REMFIRST"] = "1"
        out["host_remainder_first_%d" % rep] = med(bare, reps)
        os.environ.pop("BCOSGPU_PIPE_HEAD")
        os.environ.pop("BCOSGPU_PIPE_REMFIRST")
        out["host_default_%d" % rep] = med(bare, reps)
    out["matches"] = bool(np.array_equal(t2, st.cpu().numpy()) and np.array_equal(h, th.cpu().numpy()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
