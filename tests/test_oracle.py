"""The oracle against the reference's own golden vectors (CPU; pins the checker before it is trusted).

Mirrors bcos-crypto/test/unittests/HashTest.cpp, SignatureTest.cpp, testMerkle.cpp and the
reference-produced Merkle roots of SURVEY.md §8c.
"""
import hashlib
import struct

import numpy as np
import pytest

from conftest import load_golden


def test_hash_kats(oracle, kat):  # HashTest.cpp:59-99
    for v in kat["hash"]:
        h = oracle.keccak256 if v["hasher"] == "keccak256" else oracle.sm3
        assert h(v["msg"].encode()).hex() == v["digest"], v


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 135, 136, 137, 200, 271, 272, 1000])
def test_sm3_vs_hashlib(oracle, n):
    m = bytes((i * 37 + 11) & 0xFF for i in range(n))
    assert oracle.sm3(m) == hashlib.new("sm3", m).digest()


def test_keccak_vs_python_restatement(oracle):
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import keccak256
    for n in (0, 1, 8, 135, 136, 137, 271, 272, 273, 500):
        m = bytes((i * 13 + 5) & 0xFF for i in range(n))
        assert oracle.keccak256(m) == keccak256(m)


def test_secp256k1_kats(oracle, kat):  # SignatureTest.cpp:53-63, EVMPrecompiledTest.cpp:58-72
    for v in kat["secp256k1_pubkey"]:
        assert oracle.secp256k1_pubkey(bytes.fromhex(v["sk"])).hex() == v["pub"]
    for v in kat["secp256k1_recover"]:
        pub = oracle.secp256k1_recover(bytes.fromhex(v["hash"]), bytes.fromhex(v["sig"]))
        assert (pub is not None) == v["ok"], v
        if "address_keccak" in v:
            assert oracle.keccak256(pub)[12:].hex() == v["address_keccak"]


def test_sm2_kats(oracle, kat):  # SignatureTest.cpp:238-251
    for v in kat["sm2_pubkey"]:
        assert oracle.sm2_pubkey(bytes.fromhex(v["sk"])).hex() == v["pub"]
    for v in kat["sm2_verify"]:
        h = oracle.sm3(v["msg"].encode())
        assert (oracle.sm2_recover(h, bytes.fromhex(v["sig"])) is not None) == v["ok"]
        # without the pubkey suffix (or with any other length) SM2Crypto::recover throws
        assert oracle.sm2_recover(h, bytes.fromhex(v["sig"])[:127]) is None


def test_ecc_openssl_vectors(oracle, ecc_golden):
    for v in ecc_golden["secp256k1_recover"]:
        pub = oracle.secp256k1_recover(bytes.fromhex(v["hash"]), bytes.fromhex(v["sig"]))
        assert (pub is not None) == v["ok"]
        if v["ok"]:
            assert pub.hex() == v["pub"]
    for v in ecc_golden["sm2_verify"]:
        ok = oracle.sm2_recover(bytes.fromhex(v["hash"]), bytes.fromhex(v["sig"])) is not None
        assert ok == v["ok"]


def test_sign_roundtrip_and_negative_cases(oracle):
    """SignatureTest.cpp:107-179 / :253-302 semantics: secp recover of a wrong-hash signature succeeds
    with a different key (TxPoolTest.cpp:469-489 accepts it); SM2 rejects it."""
    rng = np.random.default_rng(7)
    for _ in range(8):
        sk, h, h2, k = (rng.bytes(32) for _ in range(4))
        pub = oracle.secp256k1_pubkey(sk)
        sig = oracle.secp256k1_sign(sk, h, k)
        assert oracle.secp256k1_recover(h, sig) == pub
        assert oracle.secp256k1_verify(pub, h, sig)
        other = oracle.secp256k1_recover(h2, sig)
        assert other is not None and other != pub
        assert not oracle.secp256k1_verify(pub, h2, sig)
        spub = oracle.sm2_pubkey(sk)
        ssig = oracle.sm2_sign(sk, h, k)
        assert ssig[64:] == spub and oracle.sm2_recover(h, ssig) == spub
        assert oracle.sm2_recover(h2, ssig) is None
        bad = bytearray(ssig); bad[5] ^= 1
        assert oracle.sm2_recover(h, bytes(bad)) is None
    v4 = bytes(64) + b"\x04"
    assert oracle.secp256k1_recover(bytes(32), v4) is None


def _bench_leaves(n):
    return np.frombuffer(b"".join(hashlib.new("sm3", struct.pack("<Q", i)).digest() for i in range(n)),
                         dtype=np.uint8).reshape(n, 32)


def test_merkle_golden(oracle, merkle_golden):
    cache = {}
    for c in merkle_golden["cases"]:
        n = c["n"]
        if n not in cache:
            cache[n] = _bench_leaves(n)
        h = oracle.SM3 if c["hasher"] == "sm3" else oracle.KECCAK256
        if c["variant"] == "old":
            assert oracle.merkle_old(h, cache[n]).hex() == c["root"], c
            continue
        root, tree = oracle.merkle(h, c["width"], cache[n], want_tree=True, nthreads=4)
        assert root.hex() == c["root"], c
        if "tree" in c:
            assert [e.tobytes().hex() for e in tree] == c["tree"]


def test_merkle_empty_throws(oracle):  # Merkle.h:172-175, testMerkle.cpp
    with pytest.raises(ValueError):
        oracle.merkle(oracle.SM3, 2, np.zeros((0, 32), dtype=np.uint8))
    assert oracle.merkle_old(oracle.SM3, np.zeros((0, 32), dtype=np.uint8)) == oracle.sm3(b"")


def test_merkle_proof_restatement(oracle):
    """The oracle's generateMerkleProof / verifyMerkleProof restatement against the reference's own
    properties (testMerkle.cpp:91-121): every leaf's proof verifies against the root, a zero hash does
    not, a proof with one entry replaced by zeros does not (when longer than 1), out of range raises,
    an empty proof raises."""
    rng = np.random.default_rng(77)
    for width in (2, 3, 16):
        for n in (1, 2, 3, 5, 17, 40):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            root = oracle.merkle(0, width, leaves)
            for i in range(n):
                proof = oracle.merkle_proof(0, width, leaves, i)
                assert oracle.merkle_verify_proof(0, proof, leaves[i].tobytes(), root)
                assert not oracle.merkle_verify_proof(0, proof, bytes(32), root)
                if len(proof) > 1:
                    bad = list(proof)
                    bad[int(rng.integers(0, len(bad)))] = bytes(32)
                    assert not oracle.merkle_verify_proof(0, bad, leaves[i].tobytes(), root)
            with pytest.raises(ValueError):
                oracle.merkle_proof(0, width, leaves, n)
            with pytest.raises(ValueError):
                oracle.merkle_verify_proof(0, [], leaves[0].tobytes(), root)


def test_merkle_bytes_vector_restatement(oracle):
    """The vector<bytes> restatement (Merkle.h:170-217 with resizeTo, Basic.h:50-61) carries the same nodes
    and root as the 32-byte-entry output vector; only the count records shrink to 4 bytes."""
    import numpy as np
    rng = np.random.default_rng(41)
    for hasher in (oracle.KECCAK256, oracle.SM3):
        for width in (2, 3, 16):
            for n in (1, 2, 3, 17, 257, 1000):
                leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
                ent = oracle.merkle_bytes_vector(hasher, width, leaves)
                root, tree = oracle.merkle(hasher, width, leaves, want_tree=True)
                assert ent[-1] == root and len(ent) == tree.shape[0]
                for e, t in zip(ent, tree):
                    assert e == (t.tobytes() if len(e) == 32 else t[:4].tobytes())
                    assert len(e) == 32 or t[4:].tobytes() == bytes(28)
                levels, m = 0, n
                while m > 1:
                    m, levels = -(-m // width), levels + 1
                assert sum(len(e) == 4 for e in ent) == levels
