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


@pytest.mark.parametrize("suite", [0, 1])
def test_standin_known_key_verify_matches_oracle(oracle, suite):
    """standin_verify_batch (the sealer-verify CPU baseline) gives the oracle's verdicts: valid, high-S
    (secp256k1 rejects), flipped bits, another key, r = 0."""
    if oracle.standin() is None:
        pytest.skip("OpenSSL stand-in not built (no /opt/conda OpenSSL)")
    rng = np.random.default_rng(21 + suite)
    n = 200
    N = (0xFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123 if suite
         else 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141)
    pubs, hs, sigs = [], [], []
    for i in range(n):
        h = rng.bytes(32)
        sk = bytes([rng.integers(1, 0x7F)]) + rng.bytes(31)
        k = bytes([rng.integers(1, 0x7F)]) + rng.bytes(31)
        if suite:
            full = oracle.sm2_sign(sk, h, k)
            sig, pub = bytearray(full[:64]), full[64:]
        else:
            s65 = oracle.secp256k1_sign(sk, h, k)
            sig, pub = bytearray(s65[:64]), oracle.secp256k1_recover(h, s65)
        kind = i % 5
        if kind == 1:
            s = int.from_bytes(sig[32:], "big")
            sig[32:] = (N - s).to_bytes(32, "big")
        elif kind == 2:
            sig[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 3 and pubs:
            pub = pubs[-1]
        elif kind == 4:
            sig[:32] = bytes(32)
        pubs.append(pub)
        hs.append(h)
        sigs.append(bytes(sig))
    P = np.frombuffer(b"".join(pubs), dtype=np.uint8).reshape(n, 64)
    H = np.frombuffer(b"".join(hs), dtype=np.uint8).reshape(n, 32)
    S = np.frombuffer(b"".join(sigs), dtype=np.uint8).reshape(n, 64)
    got = oracle.standin_verify_batch(suite, P, H, S, nthreads=4)
    if suite:
        want = [oracle.sm2_recover(hs[i], sigs[i] + pubs[i]) is not None for i in range(n)]
    else:
        want = [oracle.secp256k1_verify(pubs[i], hs[i], sigs[i]) for i in range(n)]
    assert list(got) == want
    assert all(want[0::5]) and not any(want[4::5])
