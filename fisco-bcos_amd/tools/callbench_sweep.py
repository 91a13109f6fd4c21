"""Single-call coalescing sweep (tools/callbench.cpp over the coalesced C ABI): host threads x batches
in flight (BCOSGPU_COALESCE_SLOTS), per suite, with the coalescer's phase breakdown (bcosgpu_coalesce_stats).  Writes the callbench data file (C2-size synthetic batch,
expected results from the batch path) to argv[1] and prints one JSON line per configuration."""
import json
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))

import numpy as np
import torch

import bcos_gpu
from bcos_gpu import device, synth

EXE = os.path.join(ROOT, "fisco-bcos_amd", "lib", "callbench")


def write_data(path, suite, n=8192):
    b = synth.make_batch(suite, n, seed=11 + suite)
    hashes = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    device.hash_batch(device.SM3 if suite else device.KECCAK256, b.pre, b.pre_off, hashes)
    h, s = hashes.cpu().numpy(), b.sig.view(n, b.sig_len).cpu().numpy()
    crypto = bcos_gpu.Secp256k1Crypto() if suite == 0 else bcos_gpu.SM2Crypto()
    pub, ok = crypto.recover_batch(h, s)
    with open(path, "wb") as f:
        f.write(b"BGCT" + struct.pack("<II", suite, n))
        for a in (h, s, ok.astype(np.uint8), pub if suite == 0 else s[:, 64:128]):
            f.write(np.ascontiguousarray(a, dtype=np.uint8).tobytes())


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    # argv[2]: thread counts, argv[3]: slot counts, argv[4]: BCOSGPU_COALESCE_WAIT modes (comma lists)
    ths = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 64, 256]
    sls = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [4, 8]
    waits = sys.argv[4].split(",") if len(sys.argv) > 4 else [os.environ.get("BCOSGPU_COALESCE_WAIT", "0")]
    configs = [(t, sl, 2048, w) for t in ths for sl in sls for w in waits]
    for suite in (0, 1):
        path = os.path.join(out_dir, "callbench_%d.bin" % suite)
        write_data(path, suite)
        for threads, slots, prio, wait in configs:
            calls = 1000
            env = dict(os.environ, BCOSGPU_COALESCE_SLOTS=str(slots), BCOSGPU_COALESCE_ZEROCOPY=str(prio),
                       BCOSGPU_COALESCE_WAIT=wait)
            r = subprocess.run([EXE, path, str(threads), str(calls)], capture_output=True, text=True, timeout=120,
                               env=env)
            res = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {"rc": r.returncode}
            res.update(slots=slots, zerocopy=prio, wait=int(wait), rc=r.returncode)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
