"""Writes the bench's synthetic SM2 batch (synth.make_batch(1, n)) as raw files for the tools/sm2bench
phase probe: <dir>/pre.bin (n fixed-length preimages) and <dir>/sig.bin (n x 128 bytes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bcos_gpu import synth  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
b = synth.make_batch(1, n)
b.pre.cpu().numpy().tofile(os.path.join(out, "pre.bin"))
b.sig.cpu().numpy().tofile(os.path.join(out, "sig.bin"))
print("wrote", n, "txs, preimage", b.pre.numel() // n, "bytes")
