"""The OpenSSL stand-in timed as bench.py's cpu_baseline (oracle/standin_openssl.c)
computes the same Transaction::verify results (Transaction.h:68-82) as the oracle on a signed batch
with corrupted signatures: it is a baseline of the same work, not of something easier.  CPU only."""
import os

import numpy as np
import pytest


def _batch(oracle, suite, n, seed):
    rng = np.random.default_rng(seed)
    pres, sigs = [], []
    for i in range(n):
        pre = oracle.tx_preimage(0, "chain0", "group0", 500, str(10 ** 18 + i), rng.bytes(20).hex(),
                                 rng.bytes(68), "")
        h = oracle.sm3(pre) if suite else oracle.keccak256(pre)
        sk = bytes([rng.integers(1, 0x7F)]) + rng.bytes(31)
        k = bytes([rng.integers(1, 0x7F)]) + rng.bytes(31)
        sig = bytearray(oracle.sm2_sign(sk, h, k) if suite else oracle.secp256k1_sign(sk, h, k))
        if i % 7 == 3:  # flipped bit: SM2 rejects, secp recovers another key
            sig[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        if not suite and i % 11 == 5:
            sig[64] = 4  # recid out of range
        if i % 13 == 6:
            sig = sig[:-1]  # wrong length
        pres.append(pre)
        sigs.append(bytes(sig))
    po = np.cumsum([0] + [len(p) for p in pres]).astype(np.uint64)
    so = np.cumsum([0] + [len(s) for s in sigs]).astype(np.uint64)
    return (np.frombuffer(b"".join(pres), dtype=np.uint8).copy(), po,
            np.frombuffer(b"".join(sigs), dtype=np.uint8).copy(), so)


@pytest.mark.parametrize("suite", [0, 1])
def test_standin_matches_oracle(oracle, suite):
    if oracle.standin() is None:
        pytest.skip("OpenSSL stand-in not built (no /opt/conda OpenSSL)")
    assert "OpenSSL 1.1.1" in oracle.standin_version()
    pre, po, sig, so = _batch(oracle, suite, 300, 11 + suite)
    want = oracle.tx_verify_packed(suite, pre, po, sig, so, nthreads=4)
    got = oracle.standin_tx_verify_packed(suite, pre, po, sig, so, nthreads=4)
    for w, g in zip(want, got):
        assert np.array_equal(w, g)
    assert 0 < int((want[2] == 0).sum()) < 300
