"""GPU parity for the SURVEY §8(f) rows built on the same kernels:
  - SignatureCrypto::verify with a known key, batched (sealer signatures, BlockValidator.cpp:141-182):
    secp256k1 (wedpr_secp256k1_verify: low-S, on-curve key) and SM2 (SM2Crypto.cpp:66-79);
  - the EVM ecRecover precompile (Precompiled.cpp:443-482);
  - many blocks' tx / receipt roots in one call (BlockImpl.h:111-183), incl. empty and 1-tx blocks.
All bit-exact against the oracle (tests/golden vectors pin the oracle itself).
"""
import numpy as np
import pytest

from test_gpu_ecc import N_SECP, N_SM2, _dev_sign

pytestmark = pytest.mark.gpu

P_SECP = 2**256 - 2**32 - 977


# Every kernel a verify / ecRecover batch can take (bcosgpu_set_tx_kernel_policy(split, occupancy, coop,
# field)): the automatic choice, the lane-trio kernels (sig_verify_trio26_kernel, the SM2 trio kernel over
# KeyIO, the recovery trio kernel over EcrecIO), the row kernels (coop 3: ecRecover on recover_row_kernel,
# secp256k1 known-key verify on its verify mode -- ecc_sig.hip launch_sig_verify -- and SM2 on
# sm2_verify_row_kernel), the pair kernels, the one-lane kernels at occupancy 1 and 2, and the 8 x 32-bit
# field variants.
SIG_VARIANTS = {"auto": (-1, 0, 2, 1), "trio": (1, 0, 2, 1), "row": (1, 0, 3, 1), "pair": (1, 0, 1, 1),
                "onelane_occ1": (0, 1, 2, 1), "onelane_occ2": (0, 2, 2, 1), "fe32": (-1, 0, 2, 0)}


@pytest.fixture(params=sorted(SIG_VARIANTS))
def sig_variant(request, gpu):
    gpu.set_tx_kernel_policy(*SIG_VARIANTS[request.param])
    yield request.param
    gpu.set_tx_kernel_policy()


def _keys(rng, n):
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x7F
    sk[:, 31] |= 1
    return sk


def _edit(rng, pub, h, sig, i, kind, order, other_pub):
    """kinds: 0 valid, 1 high-S, 2 wrong hash, 3 other key, 4 r/s bit flip, 5 r = 0, 6 s >= n,
    7 key off the curve, 8 key x >= p, 9 r = n."""
    if kind == 1:
        s = int.from_bytes(sig[i, 32:64].tobytes(), "big")
        sig[i, 32:64] = np.frombuffer((order - s).to_bytes(32, "big"), dtype=np.uint8)
    elif kind == 2:
        h[i, 5] ^= 0x10
    elif kind == 3:
        pub[i] = other_pub
    elif kind == 4:
        sig[i, rng.integers(0, 64)] ^= 1 << int(rng.integers(0, 8))
    elif kind == 5:
        sig[i, 0:32] = 0
    elif kind == 6:
        sig[i, 32:64] = np.frombuffer((order + int(rng.integers(0, 5))).to_bytes(32, "big") if order + 5 < 2**256
                                      else order.to_bytes(32, "big"), dtype=np.uint8)
    elif kind == 7:
        pub[i, 63] ^= 1
    elif kind == 8:
        pub[i, 0:32] = 0xFF
    elif kind == 9:
        sig[i, 0:32] = np.frombuffer(order.to_bytes(32, "big"), dtype=np.uint8)


@pytest.mark.parametrize("suite", [0, 1])
def test_verify_known_key_vs_oracle(gpu, oracle, suite, sig_variant):
    rng = np.random.default_rng(31 + suite)
    n = 2000
    sk = _keys(rng, n)
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pub, sig, ok = _dev_sign(gpu, suite, sk, h)
    assert ok.all()
    pub, sig = pub.copy(), sig.copy()
    order = N_SM2 if suite else N_SECP
    for i in range(n):
        _edit(rng, pub, h, sig, i, i % 10, order, pub[(i + 1) % n].copy())
    crypto = gpu.SM2Crypto() if suite else gpu.Secp256k1Crypto()
    stride = 128 if suite else 65
    got = crypto.verify_batch(pub, h, sig[:, :stride])
    if suite:
        want = np.array([oracle.sm2_recover(h[i].tobytes(), sig[i, :64].tobytes() + pub[i].tobytes()) is not None
                         for i in range(n)])
    else:
        want = np.array([oracle.secp256k1_verify(pub[i].tobytes(), h[i].tobytes(), sig[i, :64].tobytes())
                         for i in range(n)])
    assert np.array_equal(got, want)
    kinds = np.arange(n) % 10
    assert want[kinds == 0].all() and not want[kinds == 2].any() and not want[kinds == 3].any()
    if suite == 0:
        assert not want[kinds == 1].any()  # libsecp256k1 verify rejects high-S (recover accepts it)
    # single-call shape of SignatureCrypto::verify
    assert crypto.verify(pub[0].tobytes(), h[0].tobytes(), sig[0].tobytes())
    assert not crypto.verify(pub[2].tobytes(), h[2].tobytes(), sig[2].tobytes())


def test_ecrecover_precompile_vs_oracle(gpu, oracle, sig_variant):
    from bcos_gpu.precompiled import ec_recover, ec_recover_batch
    rng = np.random.default_rng(41)
    n = 1500
    sk = _keys(rng, n)
    h = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _, sig, ok = _dev_sign(gpu, 0, sk, h)
    inputs = []
    for i in range(n):
        v = np.zeros(32, dtype=np.uint8)
        kind = i % 6
        v[31] = 27 + int(sig[i, 64]) if kind != 1 else int(rng.integers(0, 256))
        if kind == 2:
            v[int(rng.integers(0, 31))] = int(rng.integers(1, 256))  # upper bytes of v are not read
        r, s = sig[i, 0:32].copy(), sig[i, 32:64].copy()
        if kind == 3:
            s[int(rng.integers(0, 32))] ^= 1
        if kind == 4:
            r[:] = 0
        inputs.append(h[i].tobytes() + v.tobytes() + r.tobytes() + s.tobytes())
    out, okg = ec_recover_batch(inputs)
    for i in range(n):
        want = oracle.ecrecover(inputs[i])
        assert bool(okg[i]) == (want != b""), i
        assert out[i].tobytes() == (want if want else bytes(32)), i
    assert okg.sum() > n // 2
    kat = bytes.fromhex("38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e")
    s = bytes.fromhex("789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02")
    assert ec_recover(kat + (27).to_bytes(32, "big") + kat + s) == \
        (True, bytes.fromhex("00" * 12 + "ceaccac640adf55b2028469bd36ba501f28b699d"))
    assert ec_recover(kat) == (True, b"")  # short input reads as zero-padded: v = -27 fails


@pytest.mark.parametrize("hasher,width", [(0, 2), (1, 2), (0, 16), (1, 3)])
def test_merkle_roots_batch_vs_oracle(gpu, oracle, hasher, width):
    rng = np.random.default_rng(51 + width)
    sizes = [0, 1, 2, 3, width, width + 1, 17, 255, 256, 257, 1000, 4097] + list(rng.integers(0, 3000, size=80))
    blocks = [rng.integers(0, 256, size=(int(m), 32), dtype=np.uint8) for m in sizes]  # 92 blocks: 2 chunks
    h = gpu.SM3() if hasher else gpu.Keccak256()
    got = gpu.Merkle(h, width).roots_batch(blocks)
    for b, blk in zip(got, blocks):
        want = bytes(32) if blk.shape[0] == 0 else oracle.merkle(hasher, width, blk)
        assert b == want, blk.shape


def test_receipt_and_tx_roots(gpu, oracle):
    """calculateReceiptRoot (BlockImpl.h:156-183) over receipts with logs; dataHash short-circuit."""
    rng = np.random.default_rng(61)
    for suite, hasher in ((gpu.secp256k1_suite(), 0), (gpu.sm_suite(), 1)):
        receipts, pre = [], []
        for i in range(300):
            logs = [gpu.LogEntry(address="%040x" % i, topic=[rng.bytes(32) for _ in range(int(rng.integers(0, 4)))],
                                 data=rng.bytes(int(rng.integers(0, 200)))) for _ in range(int(rng.integers(0, 3)))]
            d = gpu.TransactionReceiptData(version=0, gas_used=str(21000 + i), contract_address="",
                                           status=int(i % 3), output=rng.bytes(int(rng.integers(0, 64))),
                                           log_entries=logs, block_number=1000 + i)
            receipts.append(gpu.TransactionReceipt(data=d))
            pre.append(oracle.receipt_preimage(0, str(21000 + i), "", int(i % 3), d.output,
                                               [(l.address, l.topic, l.data) for l in logs], 1000 + i))
        receipts[7].data_hash = bytes(range(32))
        leaves = np.array([np.frombuffer(oracle.hash_(hasher, p), dtype=np.uint8) for p in pre])
        leaves[7] = np.arange(32, dtype=np.uint8)
        assert gpu.calculate_receipt_root(suite, receipts) == oracle.merkle(hasher, 2, leaves)
        assert gpu.calculate_receipt_root(suite, []) == bytes(32)
        roots = gpu.calculate_roots_batch(suite, [list(leaves[:10]), [], list(leaves)])
        assert roots == [oracle.merkle(hasher, 2, leaves[:10]), bytes(32), oracle.merkle(hasher, 2, leaves)]


@pytest.mark.parametrize("hasher,width", [(0, 2), (1, 2), (0, 16), (1, 3)])
def test_merkle_proofs_vs_oracle(gpu, oracle, hasher, width):
    """generateMerkleProof for every leaf of several trees == the oracle's restatement of Merkle.h:121-168;
    verifyMerkleProof on the GPU == the oracle's (Merkle.h:45-81), incl. the reference test's negative
    cases (testMerkle.cpp:91-121)."""
    rng = np.random.default_rng(71 + width + hasher)
    h = gpu.SM3() if hasher else gpu.Keccak256()
    mk = gpu.Merkle(h, width)
    for n in (1, 2, 3, width, width + 1, 17, 100, 257):
        leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        root = oracle.merkle(hasher, width, leaves)
        got = mk.generate_merkle_proofs(leaves, list(range(n)))
        want = [oracle.merkle_proof(hasher, width, leaves, i) for i in range(n)]
        assert got == want, n
        proofs, hashes, expect = [], [], []
        for i in range(n):
            proofs.append(got[i]); hashes.append(leaves[i].tobytes()); expect.append(True)
            proofs.append(got[i]); hashes.append(bytes(32)); expect.append(False)
            if len(got[i]) > 1:
                bad = list(got[i])
                bad[int(rng.integers(0, len(bad)))] = bytes(32)
                proofs.append(bad); hashes.append(leaves[i].tobytes())
                expect.append(oracle.merkle_verify_proof(hasher, bad, leaves[i].tobytes(), root))
        ok = mk.verify_merkle_proofs(proofs, hashes, [root] * len(proofs))
        assert list(ok) == expect
        assert mk.verify_merkle_proof(got[0], leaves[0].tobytes(), root)
        assert mk.generate_merkle_proof(leaves, leaves[n - 1].tobytes()) == want[int(np.nonzero(
            (leaves == leaves[n - 1]).all(axis=1))[0][0])]
        with pytest.raises(ValueError):
            mk.generate_merkle_proofs(leaves, [n])
        with pytest.raises(ValueError):
            mk.verify_merkle_proof([], leaves[0].tobytes(), root)
    with pytest.raises(ValueError):
        mk.generate_merkle_proof(rng.integers(0, 256, size=(4, 32), dtype=np.uint8), bytes(32))
