"""The row kernel (csrc/ecc_row.hip): secp256k1 public-key recovery with the GLV chains on row-spread
field elements (csrc/fe_row.h, csrc/ec_row.h), one signature per workgroup -- the automatic choice for
batches of up to a few hundred signatures (coalesced single recover() calls, TxValidator.cpp:27-69; a
block's ecRecover calls), forced here with bcosgpu_set_tx_kernel_policy(1, 0, 3, 1).  Against the oracle
(libsecp256k1 semantics, Secp256k1Crypto.cpp:79-93): random and edge signatures, and crafted scalars that
drive the chains and the final additions into their special cases -- u1 = 0 (the comb part at infinity),
u2 = +-c for small c (one GLV half zero: a chain that stays at infinity), Q = infinity (sR = eG, the
recovery fails) and u1 G = u2 R (the last addition is a doubling).  The fused Transaction::verify and
ecRecover paths take the same kernel in test_gpu_ecc.py / test_gpu_verify.py's variant lists."""
import numpy as np
import pytest

from test_gpu_ecc import N_SECP, _dev_sign, _mutate

pytestmark = pytest.mark.gpu

ROW = (1, 0, 3, 1)


@pytest.fixture
def row_policy(gpu):
    gpu.set_tx_kernel_policy(*ROW)
    yield
    gpu.set_tx_kernel_policy()


def _check(gpu, oracle, h, sig):
    pub, addr, okg = gpu.Secp256k1Crypto().recover_batch(h, sig, want_address=True)
    want_pub, want_ok = oracle.secp256k1_recover_batch(h, sig, nthreads=8)
    assert np.array_equal(okg, want_ok)
    assert np.array_equal(pub[want_ok], want_pub[want_ok])
    assert not pub[~want_ok].any() and not addr[~want_ok].any()
    for i in np.nonzero(want_ok)[0]:
        assert addr[i].tobytes() == oracle.keccak256(want_pub[i].tobytes())[12:], i
    return want_ok


@pytest.mark.parametrize("n", [1, 7, 257, 1000])
def test_row_recover_random_and_edge(gpu, oracle, row_policy, n):
    """Valid signatures and the nine mutation kinds of test_gpu_ecc (bit flips, v out of range, random
    r || s, r = n, s = 0, r >= n, small r with v = 2 / 3 -- x = r + n) at 1, 7, 257 (one more than a
    round on 256 CUs) and 1,000 signatures, with zero and all-ones digests."""
    rng = np.random.default_rng(0x50 + n)
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x7F
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    h[: max(1, n // 20)] = 0
    h[n // 20: n // 10] = 0xFF
    _, sig, _ = _dev_sign(gpu, 0, sk, h)
    arr = np.array([np.frombuffer(_mutate(rng, sig[i].tobytes(), (i % 9) if n > 1 else 0), dtype=np.uint8)
                    for i in range(n)])
    ok = _check(gpu, oracle, h, arr)
    if n >= 257:
        assert ok.sum() > n // 4 and (~ok).sum() > n // 10


def _b32(x):
    return np.frombuffer(int(x % N_SECP).to_bytes(32, "big"), dtype=np.uint8)


def test_row_recover_crafted_scalars(gpu, oracle, row_policy):
    """R = k G for a known nonce k (so r, v follow from k), then s and e chosen to make: u1 = 0 (e = 0,
    e = n), u2 = c and u2 = -c for c = 1..12 (k2 = 0 after the GLV split), Q = O (e = s k: the
    recovery fails), u1 G = u2 R (e = -s k: the final addition doubles)."""
    rng = np.random.default_rng(0xC4AF)
    hs, sigs = [], []
    for t in range(40):
        k = int.from_bytes(rng.bytes(32), "big") % N_SECP or 1
        R = oracle.secp256k1_pubkey(k.to_bytes(32, "big"))
        rx, ry = int.from_bytes(R[:32], "big"), int.from_bytes(R[32:], "big")
        if rx >= N_SECP:
            continue
        r, v = rx, ry & 1
        s = int.from_bytes(rng.bytes(32), "big") % N_SECP or 1
        cases = []
        c = 1 + t % 12
        cases.append((0, s))                         # u1 = 0
        cases.append((N_SECP, s))                    # e = n -> e mod n = 0
        cases.append((int.from_bytes(rng.bytes(32), "big"), r * c))             # u2 = c
        cases.append((int.from_bytes(rng.bytes(32), "big"), r * (N_SECP - c)))  # u2 = -c
        cases.append((s * k, s))                     # s R = e G: Q at infinity
        cases.append((-s * k, s))                    # u1 G = u2 R: Q = 2 u1 G
        for e, ss in cases:
            ss %= N_SECP
            if ss == 0:
                continue
            hs.append(np.frombuffer(int(e % 2**256).to_bytes(32, "big"), dtype=np.uint8) if e == N_SECP
                      else _b32(e))
            sigs.append(np.concatenate([_b32(r), _b32(ss), np.array([v], dtype=np.uint8)]))
    h, sig = np.array(hs), np.array(sigs)
    ok = _check(gpu, oracle, h, sig)
    assert (~ok).sum() >= 20  # the Q = O cases
    assert ok.sum() >= 100


# ------------------------------------------------------------------ SM2 (sm2_verify_row_kernel)
N_SM2 = 0xFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123


@pytest.mark.parametrize("n", [1, 7, 300])
def test_row_sm2_verify_random_and_edge(gpu, oracle, row_policy, n):
    """SM2Crypto::recover / verify with the embedded key (r || s || pub) through the SM2 row kernel:
    valid signatures, bit flips, a wrong hash, r = n, s = 0, r + s = n (t = 0), a key with x >= p, a key
    off the curve, r + s = n - 2 and n - 4 (t near n: the chain's last addition meets its doubling /
    infinity cases), against the oracle's verdicts and addresses."""
    rng = np.random.default_rng(0x5A + n)
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x7F
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _, sig, _ = _dev_sign(gpu, 1, sk, h)
    sig = sig.copy()
    for i in range(n if n > 1 else 0):
        kind = i % 10
        if kind == 1:
            sig[i, rng.integers(0, 128)] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            h[i, 0] ^= 1
        elif kind == 3:
            sig[i, 0:32] = np.frombuffer(N_SM2.to_bytes(32, "big"), dtype=np.uint8)
        elif kind == 4:
            sig[i, 32:64] = 0
        elif kind in (5, 8, 9):  # r + s = n, n - 2, n - 4
            r = int.from_bytes(sig[i, 0:32].tobytes(), "big")
            off = {5: 0, 8: 2, 9: 4}[kind]
            sig[i, 32:64] = np.frombuffer(((N_SM2 - off - r) % N_SM2).to_bytes(32, "big"), dtype=np.uint8)
        elif kind == 6:
            sig[i, 64:96] = 0xFF
        elif kind == 7:
            sig[i, 127] ^= 1
    _, addr, okg = gpu.SM2Crypto().recover_batch(h, sig, want_address=True)
    want = oracle.sm2_verify_batch(h, sig, nthreads=8)
    assert np.array_equal(okg, want)
    assert not addr[~want].any()
    for i in np.nonzero(want)[0]:
        assert addr[i].tobytes() == oracle.sm3(sig[i, 64:].tobytes())[12:], i
    if n >= 300:  # kind 0 (one in ten) is the valid case; every other kind is rejected
        assert want.sum() >= n // 12 and (~want).sum() >= n // 2
