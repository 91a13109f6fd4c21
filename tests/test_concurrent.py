"""Concurrent single-signature calls through the drop-in SignatureCrypto classes (include/bcos_gpu_crypto.hpp):
the reference's admission pattern -- TxPool's hardware_concurrency submitter threads (TxPool.h:48-49)
each running TxValidator::verify -> Transaction::verify -> SignatureCrypto::recover once per tx
(TxValidator.cpp:56, Transaction.h:68-82) -- 64 threads x 2,000 and 256 threads x 500 calls per suite
(256: the reference host's hardware_concurrency; past 128 callers the coalescer caps its batches in
flight, and most arrivals take the lock-free path), every result bit-identical to the oracle.  The
engine coalesces the calls into shared launches (csrc/coalesce.hip)."""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from test_cpp_adapter import LIBDIR, ROOT
from test_gpu_ecc import _dev_sign, _mutate, _mutate_sm2

ITEMS = 16384


def _build(tmp_path):
    exe = str(tmp_path / "concurrent_test")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "tests", "cpp", "mirror"),
                    "-I" + os.path.join(ROOT, "include"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "concurrent_test.cpp"), "-L" + LIBDIR, "-lbcosgpu",
                    "-Wl,-rpath," + LIBDIR, "-lpthread"], check=True)
    return exe


def test_concurrent_test_compiles(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2  # usage


def _write(path, suite, h, sig, ok, pub):
    with open(path, "wb") as f:
        f.write(b"BGCT" + struct.pack("<II", suite, h.shape[0]))
        for a in (h, sig, ok.astype(np.uint8), pub):
            f.write(np.ascontiguousarray(a, dtype=np.uint8).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("threads,calls", [(64, 2000), (256, 500)])
@pytest.mark.parametrize("suite", [0, 1])
def test_concurrent_single_recover_calls(gpu, oracle, tmp_path, suite, threads, calls):
    rng = np.random.default_rng(500 + suite)
    sk = rng.integers(0, 256, size=(ITEMS, 32), dtype=np.uint8)
    sk[:, 0] &= 0x7F
    h = rng.integers(0, 256, size=(ITEMS, 32), dtype=np.uint8)
    _, sig, _ = _dev_sign(gpu, suite, sk, h)
    # a quarter of the calls carry the reference's edge cases (bad v, r = n, s = 0, flipped bits, ...)
    sig = np.array([np.frombuffer((_mutate(rng, sig[i].tobytes(), i % 9) if suite == 0
                                   else _mutate_sm2(rng, sig[i].tobytes(), i % 8)) if i % 4 == 1 else sig[i].tobytes(),
                                  dtype=np.uint8) for i in range(ITEMS)])
    if suite == 0:
        pub, ok = oracle.secp256k1_recover_batch(h, sig, nthreads=16)
    else:
        ok = oracle.sm2_verify_batch(h, sig, nthreads=16)
        pub = sig[:, 64:128]
    assert 0 < ok.sum() < ITEMS
    data = str(tmp_path / "calls.bin")
    _write(data, suite, h, sig, ok, pub)
    exe = _build(tmp_path)
    r = subprocess.run([exe, data, str(threads), str(calls)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatches"] == 0 and res["engine_errors"] == 0 and res["calls"] == threads * calls
    print(res)
