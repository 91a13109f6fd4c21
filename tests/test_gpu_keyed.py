"""GPU parity of verification against REGISTERED keys (csrc/ecc_keyed.hip): the sealer path of
BlockValidator::checkSignatureList (bcos-pbft/.../BlockValidator.cpp:141-182) and
PBFTCacheProcessor::checkPrecommitWeight (PBFTCacheProcessor.cpp:795-821) -> SignatureCrypto::verify
(Secp256k1Crypto.cpp:51-63, SM2Crypto.cpp:66-79), whose keys are the consensus node list.

Every verdict is compared with the oracle (oracle/ec.c: libsecp256k1 ecdsa_verify semantics with low-S;
sm2_do_verify), through the device-resident slot API, the coalesced host calls once the keys are
registered or promoted, and SM2 recover with a registered embedded key.  The registered-key kernel sums
16 partial sums per signature with complete additions; signatures whose partial sums coincide (P = Q)
or cancel (P = -Q) are built here from chosen private keys (a key's owner can do the same) and must
verify exactly as the oracle says."""
import numpy as np
import pytest

from test_gpu_ecc import N_SECP, N_SM2, _dev_sign
from test_gpu_verify import _edit, _keys

pytestmark = pytest.mark.gpu

P_SECP = 2**256 - 2**32 - 977
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def _add(P, Q):
    """secp256k1 affine addition over Python integers (None = infinity)."""
    if P is None:
        return Q
    if Q is None:
        return P
    (x1, y1), (x2, y2) = P, Q
    if x1 == x2 and (y1 + y2) % P_SECP == 0:
        return None
    if P == Q:
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P_SECP) % P_SECP
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P_SECP) % P_SECP
    x3 = (lam * lam - x1 - x2) % P_SECP
    return x3, (lam * (x1 - x3) - y1) % P_SECP


def _mul(k, P=(GX, GY)):
    R = None
    for bit in bin(k % N_SECP)[2:]:
        R = _add(R, R)
        if bit == "1":
            R = _add(R, P)
    return R


def _pub_bytes(P):
    return P[0].to_bytes(32, "big") + P[1].to_bytes(32, "big")


def _crafted(d, u1, u2):
    """A signature (hash e, r, s) whose verification computes u1 G + u2 P for P = d G, or None when the
    resulting s is high (libsecp256k1 rejects it) or degenerate.  The verdict is valid by construction."""
    R = _mul(u1 + u2 * d)
    if R is None:
        return None
    r = R[0] % N_SECP
    s = r * pow(u2, -1, N_SECP) % N_SECP
    if r == 0 or s == 0 or s > N_SECP // 2:
        return None
    e = u1 * s % N_SECP
    return e.to_bytes(32, "big"), r.to_bytes(32, "big") + s.to_bytes(32, "big")


def _exceptional_cases():
    """(pub, hash, sig64, label): the registered-key kernel's lane L holds 2^(16L) (c_L d + w_L) G, c_L / w_L
    the 16-bit windows of u2 / u1 (the default 16-bit G comb).  Lanes 0 and 1 equal (level-1 doubling),
    opposite (level-1 cancellation, the total kept nonzero by lane 2), lanes {0, 1} equal to lanes
    {2, 3} (level-2 doubling), and a total of infinity (must fail)."""
    out = []
    # (label, c0 -> (d, u1)); u2 = c0 (window 0 only).  The sum u1 + u2 d, hence r, is fixed per label, so
    # c0 varies s = r / c0 until it is low
    specs = [("dbl1", lambda c0: ((2**16 - 5) * pow(c0, -1, N_SECP) % N_SECP, 5 + 2**16)),  # c0 d + w0 = 2^16 w1
             ("neg1", lambda c0: ((-2**16 - 5) * pow(c0, -1, N_SECP) % N_SECP, 5 + 2**16 + 2**32)),  # = -2^16 w1
             ("dbl2", lambda c0: ((2**32 - 5) * pow(c0, -1, N_SECP) % N_SECP, 5 + 2**32))]  # c0 d + w0 = 2^32 w2
    for label, f in specs:
        found = 0
        for c0 in range(1, 200):
            d, u1 = f(c0)
            c = _crafted(d, u1, c0)
            if c is not None:
                out.append((_pub_bytes(_mul(d)), c[0], c[1], label))
                found += 1
                if found == 3:
                    break
    # u1 G + u2 P = infinity: u1 = -u2 d
    d, u2 = 0x1234567, 5
    u1 = (-u2 * d) % N_SECP
    s = 7
    r = u2 * s % N_SECP
    out.append((_pub_bytes(_mul(d)), (u1 * s % N_SECP).to_bytes(32, "big"), r.to_bytes(32, "big") + s.to_bytes(32, "big"),
                "inf"))
    return out


def _oracle_verify(oracle, suite, pub, h, sig):
    if suite:
        return oracle.sm2_recover(h, sig[:64] + pub) is not None
    return oracle.secp256k1_verify(pub, h, sig[:64])


def _wait_built(gpu, suite, target, timeout=10.0):
    """Promotion builds run asynchronously (ecc_keyed.hip keyed_slots): poll the cache until `target` tables
    have been built and published."""
    import time
    t0 = time.monotonic()
    while gpu.key_cache_info(suite)["built"] < target:
        assert time.monotonic() - t0 < timeout, "promotion build not published"
        time.sleep(0.001)
    return gpu.key_cache_info(suite)


def _keyed_dev(suite, slots, h, sig):
    import torch
    from bcos_gpu import device
    n = len(slots)
    d_slots = torch.from_numpy(np.ascontiguousarray(slots, dtype=np.int32)).cuda()
    d_h = torch.from_numpy(np.ascontiguousarray(h, dtype=np.uint8)).cuda()
    d_s = torch.from_numpy(np.ascontiguousarray(sig, dtype=np.uint8)).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    device.verify_keyed(suite, d_slots, d_h, d_s, ok)
    torch.cuda.synchronize()
    return ok.cpu().numpy().astype(bool)


@pytest.mark.parametrize("suite", [0, 1])
def test_registered_keys_vs_oracle(gpu, oracle, suite):
    """48 registered keys (two of them invalid: off the curve, x >= p), 1,500 signatures over them with the
    verify suite's edits (valid, high-S, wrong hash, another registered key, bit flips, r = 0, s >= n,
    r = n, e = 0): the device slot API and the coalesced host batch both equal the oracle, the host batch
    on the registered-key kernel."""
    rng = np.random.default_rng(501 + suite)
    nk, n = 48, 1500
    sk = _keys(rng, nk)
    pub, _, ok = _dev_sign(gpu, suite, sk, np.zeros((nk, 32), dtype=np.uint8))
    assert ok.all()
    pub = pub.copy()
    pub[nk - 2, 63] ^= 1   # off the curve
    pub[nk - 1, 0:32] = 0xFF  # x >= p
    slots = gpu.register_keys(suite, pub)
    assert (slots >= 0).all() and len(set(slots.tolist())) == nk
    assert (gpu.register_keys(suite, pub) == slots).all()  # registering again is a lookup
    who = rng.integers(0, nk - 2, size=n)
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    h[7] = 0  # e = 0: u1 = 0
    _, sig, ok = _dev_sign(gpu, suite, sk[who], h)
    assert ok.all()
    sig = sig.copy()
    order = N_SM2 if suite else N_SECP
    kp = pub[who].copy()
    for i in range(n):
        kind = i % 10
        if kind in (7, 8):  # the invalid registered keys
            who[i] = nk - 2 if kind == 7 else nk - 1
            kp[i] = pub[who[i]]
        elif kind == 3:  # another registered key
            who[i] = (who[i] + 1) % (nk - 2)
            kp[i] = pub[who[i]]
        else:
            _edit(rng, kp, h, sig, i, kind, order, None)
    want = np.array([_oracle_verify(oracle, suite, kp[i].tobytes(), h[i].tobytes(), sig[i].tobytes())
                     for i in range(n)])
    assert want[np.arange(n) % 10 == 0].all() and not want[np.arange(n) % 10 == 7].any()
    got = _keyed_dev(suite, slots[who], h, sig)
    assert np.array_equal(got, want)
    before = gpu.key_cache_info(suite)
    crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
    assert np.array_equal(crypto.verify_batch(kp, h, sig), want)
    after = gpu.key_cache_info(suite)
    assert after["keyed"] - before["keyed"] >= n  # the coalesced batch took the registered-key kernel
    # unregistered slots fail
    bad = _keyed_dev(suite, np.array([-1, 1 << 20], dtype=np.int32), h[:2], sig[:2])
    assert not bad.any()


def test_registered_key_exceptional_additions(gpu, oracle):
    """secp256k1 signatures whose partial sums in the registered-key kernel coincide or cancel (crafted from
    chosen private keys, valid by construction) and one whose total is infinity: same verdicts as the oracle
    on the keyed path and on the generic path."""
    cases = _exceptional_cases()
    labels = {c[3] for c in cases}
    assert {"dbl1", "neg1", "dbl2", "inf"} <= labels, labels
    pubs = np.array([np.frombuffer(c[0], dtype=np.uint8) for c in cases])
    h = np.array([np.frombuffer(c[1], dtype=np.uint8) for c in cases])
    sig = np.array([np.frombuffer(c[2], dtype=np.uint8) for c in cases])
    want = np.array([oracle.secp256k1_verify(c[0], c[1], c[2]) for c in cases])
    assert want[[c[3] != "inf" for c in cases]].all() and not want[[c[3] == "inf" for c in cases]].any()
    slots = gpu.register_keys(0, pubs)
    assert (slots >= 0).all()
    assert np.array_equal(_keyed_dev(0, slots, h, sig), want)
    assert np.array_equal(gpu.Secp256k1Crypto().verify_batch(pubs, h, sig), want)
    # the generic known-key kernels on the same owner-crafted cases: keys forgotten, then the row verify
    # kernel (policy coop 3) and the lane-trio kernel (coop 2), each checked to have left the keyed path
    for policy in ((1, 0, 3, 1), (1, 0, 2, 1)):
        gpu.clear_keys(0)
        gpu.set_tx_kernel_policy(*policy)
        try:
            k0 = gpu.key_cache_info(0)["keyed"]
            assert np.array_equal(gpu.Secp256k1Crypto().verify_batch(pubs, h, sig), want), policy
            assert gpu.key_cache_info(0)["keyed"] == k0, policy
        finally:
            gpu.set_tx_kernel_policy()
    gpu.clear_keys(0)


def test_promotion_single_calls_and_sm2_recover(gpu, oracle):
    """Keys seen in three calls are promoted (BCOSGPU_KEY_PROMOTE, default 3): the third batch starts their
    table build (asynchronous; that batch itself stays on the generic kernels), and the batches and single
    SignatureCrypto::verify calls after it is published run on the registered-key kernel with the oracle's
    verdicts; SM2
    recover (SM2Crypto::recover, embedded key) over registered keys returns the same addresses as the
    generic path."""
    rng = np.random.default_rng(777)
    for suite in (0, 1):
        crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
        nk = 7
        sk = _keys(rng, nk)
        h = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
        pub, sig, ok = _dev_sign(gpu, suite, sk, h)
        assert ok.all()
        want = np.ones(nk, dtype=bool)
        i0 = gpu.key_cache_info(suite)
        assert np.array_equal(crypto.verify_batch(pub, h, sig), want)   # first sighting: generic
        assert np.array_equal(crypto.verify_batch(pub, h, sig), want)   # second: generic
        assert gpu.key_cache_info(suite)["built"] == i0["built"]
        assert np.array_equal(crypto.verify_batch(pub, h, sig), want)   # third: promoted
        i1 = _wait_built(gpu, suite, i0["built"] + nk)
        assert i1["built"] - i0["built"] == nk and i1["keys"] - i0["keys"] == nk
        assert np.array_equal(crypto.verify_batch(pub, h, sig), want)   # after the build: keyed
        assert gpu.key_cache_info(suite)["keyed"] - i1["keyed"] >= nk
        i1 = gpu.key_cache_info(suite)
        for i in range(nk):
            assert crypto.verify(pub[i].tobytes(), h[i].tobytes(), sig[i].tobytes())
            bad = bytearray(sig[i].tobytes())
            bad[3] ^= 0x40
            assert not crypto.verify(pub[i].tobytes(), h[i].tobytes(), bytes(bad))
        assert gpu.key_cache_info(suite)["keyed"] - i1["keyed"] >= 2 * nk
    # SM2 recover with registered embedded keys: verdicts and SM3 addresses
    n = 300
    sk = _keys(rng, 12)
    who = rng.integers(0, 12, size=n)
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pub, sig, ok = _dev_sign(gpu, 1, sk[who], h)
    sig = sig.copy()
    sig[::5, 9] ^= 4
    gpu.register_keys(1, pub)
    crypto = gpu.SM2Crypto()
    k0 = gpu.key_cache_info(1)["keyed"]
    _, got_addr, got_ok = crypto.recover_batch(h, sig, want_address=True)
    assert gpu.key_cache_info(1)["keyed"] - k0 >= n
    want_ok = oracle.sm2_verify_batch(h, sig)
    assert np.array_equal(got_ok, want_ok)
    for i in np.nonzero(want_ok)[0]:
        assert got_addr[i].tobytes() == oracle.sm3(pub[i].tobytes())[12:]


def test_clear_and_reregister(gpu, oracle):
    """bcosgpu_clear_keys (a consensus membership change) forgets every key; registering another set reuses
    the slots; the forgotten keys' signatures then verify on the generic kernels and the new keys' on the
    registered-key kernel, every verdict equal to the oracle's."""
    rng = np.random.default_rng(4242)
    for suite in (0, 1):
        crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
        sk_a, sk_b = _keys(rng, 5), _keys(rng, 5)
        h = rng.integers(0, 256, size=(5, 32), dtype=np.uint8)
        pa, sa, _ = _dev_sign(gpu, suite, sk_a, h)
        pb, sb, _ = _dev_sign(gpu, suite, sk_b, h)
        sa, sb = sa.copy(), sb.copy()
        sa[0, 7] ^= 1
        sb[1, 9] ^= 2
        want_a = np.array([_oracle_verify(oracle, suite, pa[i].tobytes(), h[i].tobytes(), sa[i].tobytes())
                           for i in range(5)])
        want_b = np.array([_oracle_verify(oracle, suite, pb[i].tobytes(), h[i].tobytes(), sb[i].tobytes())
                           for i in range(5)])
        slots_a = gpu.register_keys(suite, pa)
        assert np.array_equal(crypto.verify_batch(pa, h, sa), want_a)
        gpu.clear_keys(suite)
        assert gpu.key_cache_info(suite)["keys"] == 0
        slots_b = gpu.register_keys(suite, pb)
        assert sorted((slots_b & 0xFFFF).tolist()) == list(range(5))  # table indices restart: reused
        assert (slots_a >= 0).all() and not set(slots_a.tolist()) & set(slots_b.tolist())  # ids do not
        # an id from before the clear names an old generation: it fails in the kernel even though its index
        # now holds one of the new keys' tables (B's valid signatures through A's ids stay rejected)
        assert not _keyed_dev(suite, slots_a, h, sb).any()
        assert not _keyed_dev(suite, slots_a, h, sa).any()
        k0 = gpu.key_cache_info(suite)
        assert np.array_equal(crypto.verify_batch(pa, h, sa), want_a)   # forgotten: generic
        k1 = gpu.key_cache_info(suite)
        assert k1["keyed"] == k0["keyed"]
        assert np.array_equal(crypto.verify_batch(pb, h, sb), want_b)   # registered: keyed
        assert gpu.key_cache_info(suite)["keyed"] - k1["keyed"] == 5
        assert np.array_equal(_keyed_dev(suite, slots_b, h, sb), want_b)


def test_promotion_counts_calls_not_occurrences(gpu, oracle):
    """A key repeated within one call counts once toward promotion (three copies in one batch promote
    nothing), and SM2 recover -- admission, whose key is the sender's own, embedded in the signature --
    never promotes, however often a key recurs; verdicts equal the oracle's throughout."""
    rng = np.random.default_rng(99)
    for suite in (0, 1):
        gpu.clear_keys(suite)
        crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
        sk = _keys(rng, 2)
        h = rng.integers(0, 256, size=(2, 32), dtype=np.uint8)
        pub, sig, ok = _dev_sign(gpu, suite, sk, h)
        assert ok.all()
        rep = np.array([0, 0, 0, 1, 1, 1])
        b0 = gpu.key_cache_info(suite)["built"]
        assert crypto.verify_batch(pub[rep], h[rep], sig[rep]).all()
        assert crypto.verify_batch(pub[rep], h[rep], sig[rep]).all()
        assert gpu.key_cache_info(suite)["built"] == b0  # two calls: not yet, despite six occurrences
        if suite == 1:  # SM2 recover with the same embedded keys, many times: lookups only
            for _ in range(4):
                _, addr, okr = crypto.recover_batch(h[rep], sig[rep], want_address=True)
                assert okr.all()
            assert gpu.key_cache_info(suite)["built"] == b0
        assert crypto.verify_batch(pub[rep], h[rep], sig[rep]).all()  # third named call: promoted
        assert _wait_built(gpu, suite, b0 + 2)["built"] - b0 == 2
        gpu.clear_keys(suite)


def test_promotion_under_concurrent_calls(gpu, oracle):
    """Promotion builds run asynchronously (ecc_keyed.hip keyed_slots: one build in flight, published when
    its event completes): 24 threads make single SignatureCrypto::verify calls over 48 keys -- each key
    seen many times, so builds start, complete and publish while other threads look the same keys up --
    and a registration of half the keys (which waits for a build in flight) lands in the middle.  Every verdict equals the expected one (1 in 4 signatures corrupted), every
    key ends up with exactly one table, and the registered keys' ids name published tables."""
    import threading
    rng = np.random.default_rng(2468)
    for suite in (0, 1):
        gpu.clear_keys(suite)
        crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
        nk = 48
        sk = _keys(rng, nk)
        h = rng.integers(0, 256, size=(nk, 32), dtype=np.uint8)
        pub, sig, ok = _dev_sign(gpu, suite, sk, h)
        assert ok.all()
        sig = sig.copy()
        bad = np.arange(nk) % 4 == 3
        sig[bad, 5] ^= 0x10
        want = np.array([_oracle_verify(oracle, suite, pub[i].tobytes(), h[i].tobytes(), sig[i].tobytes())
                         for i in range(nk)])
        assert not want[bad].any() and want[~bad].all()
        b0 = gpu.key_cache_info(suite)["built"]
        wrong, errors = [], []
        start = threading.Barrier(25)

        def caller(t):
            try:
                start.wait()
                for j in range(60):
                    i = (j * 7 + t * 5) % nk
                    if crypto.verify(pub[i].tobytes(), h[i].tobytes(), sig[i].tobytes()) != bool(want[i]):
                        wrong.append((t, j, i))
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(repr(e))

        th = [threading.Thread(target=caller, args=(t,)) for t in range(24)]
        for x in th:
            x.start()
        start.wait()
        slots = gpu.register_keys(suite, pub[::2])
        for x in th:
            x.join()
        assert not errors and not wrong, (errors, wrong[:5])
        assert (slots >= 0).all()
        gpu.register_keys(suite, pub[:1])  # registered already: waits for a promotion build still in flight
        info = gpu.key_cache_info(suite)
        assert info["keys"] == info["built"] - b0 <= nk
        assert np.array_equal(_keyed_dev(suite, slots, h[::2], sig[::2]), want[::2])
        assert np.array_equal(crypto.verify_batch(pub, h, sig), want)
        gpu.clear_keys(suite)
