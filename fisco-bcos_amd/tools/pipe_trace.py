"""A few host-pointer tx batches (bcosgpu_tx_verify_batch) to trace under rocprofv3 --kernel-trace
--memory-copy-trace: shows whether chunk uploads overlap the previous chunk's kernel (txpipe.hip).
Usage: python pipe_trace.py N REPS [devset]  (devset: the C4 block through bcosgpu_block_verify_multi on
{0, 0}, width-2 root, as bench.py's devset leg; 50 ms idle between repetitions).  GPU tool."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import time  # noqa: E402

import numpy as np  # noqa: E402

import bcos_gpu  # noqa: E402
from bcos_gpu import synth  # noqa: E402
from bcos_gpu._lib import check, lib  # noqa: E402
from bcos_gpu.crypto import _ptr  # noqa: E402


def main():
    n, reps = int(sys.argv[1]), int(sys.argv[2])
    bcos_gpu.ensure_device(0)
    b = synth.make_batch(0, n, seed=0xC2)
    pre = np.ascontiguousarray(b.pre.cpu().numpy())
    po = np.ascontiguousarray(b.pre_off.cpu().numpy().astype(np.uint64))
    sg = np.ascontiguousarray(b.sig.cpu().numpy())
    so = np.ascontiguousarray(b.sig_off.cpu().numpy().astype(np.uint64))
    h, sd, st = np.zeros((n, 32), np.uint8), np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)
    for _ in range(reps):
        if "devset" in sys.argv:
            from bcos_gpu import tx
            tx.verify_packed_multi([0, 0], bcos_gpu.secp256k1_suite(), pre, po, sg, so, width=2, out=(h, sd, st))
            time.sleep(0.05)
        else:
            check(lib().bcosgpu_tx_verify_batch(0, _ptr(pre), _ptr(po), _ptr(sg), _ptr(so), n, _ptr(h), _ptr(sd),
                                                _ptr(st)))
    print("done", int((st == 0).sum()))


if __name__ == "__main__":
    main()
