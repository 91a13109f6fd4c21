"""Host-side mirror of the reference's crypto interfaces, backed by the HIP engine.

Mirrors (same names, argument meaning and error behaviour):
  bcos::crypto::Hash / Keccak256 / SM3         bcos-crypto/bcos-crypto/interfaces/crypto/Hash.h:37-72,
                                               hash/Keccak256.h:39-51, hash/SM3.h:39-50
  bcos::crypto::SignatureCrypto::recover/verify interfaces/crypto/Signature.h:40-58
    Secp256k1Crypto                            signature/secp256k1/Secp256k1Crypto.{h,cpp}
    SM2Crypto / FastSM2Crypto                  signature/sm2/SM2Crypto.cpp:66-92, fastsm2/FastSM2Crypto.h
  bcos::crypto::merkle::Merkle<Hasher,width>   merkle/Merkle.h:36-262 (generateMerkle :170-208)
  bcos::protocol::calculateMerkleProofRoot     bcos-protocol/bcos-protocol/ParallelMerkleProof.cpp:32-69
  bcos::crypto::CryptoSuite::calculateAddress  interfaces/crypto/CryptoSuite.h:56-59
Single-item calls keep the reference's exception semantics (recover raises InvalidSignature, an empty
Merkle input raises ValueError like std::invalid_argument); *_batch calls return per-item verdicts.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, ensure_device, lib


class InvalidSignature(Exception):
    """bcos::crypto::InvalidSignature (signature/Exceptions.h)."""


def _ptr(a):
    """the array's data address as an int (every ABI pointer parameter is declared c_void_p, which takes
    one; ~2 us cheaper per argument than ctypes.data_as on the host-pointer batch calls)"""
    return a.__array_interface__["data"][0]


def _u8(a, shape=None):
    a = np.ascontiguousarray(np.frombuffer(a, dtype=np.uint8) if isinstance(a, (bytes, bytearray)) else a,
                             dtype=np.uint8)
    return a if shape is None else a.reshape(shape)


def pack_messages(msgs):
    """list[bytes] -> (flat uint8 array, uint64 offsets[n+1])"""
    offsets = np.zeros(len(msgs) + 1, dtype=np.uint64)
    if msgs:
        offsets[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
    data = np.frombuffer(b"".join(msgs), dtype=np.uint8) if msgs else np.zeros(0, dtype=np.uint8)
    return np.ascontiguousarray(data), offsets


class Hash:
    """bcos::crypto::Hash: hash(bytesConstRef) -> h256 (Hash.h:44)."""
    HASH_SIZE = 32
    kind = None

    def hash(self, data: bytes) -> bytes:
        return self.hash_batch([bytes(data)])[0]

    def hash_batch(self, msgs):
        out = self.hash_packed(*pack_messages(list(msgs)))
        return [out[i].tobytes() for i in range(len(msgs))]

    def hash_packed(self, data, offsets):
        """data: uint8[...], offsets: uint64[n+1] -> uint8[n, 32]"""
        ensure_device()
        n = len(offsets) - 1
        out = np.zeros((n, 32), dtype=np.uint8)
        if n:
            d = data if len(data) else np.zeros(1, dtype=np.uint8)
            check(lib().bcosgpu_hash_batch(self.kind, _ptr(d), _ptr(offsets), n, _ptr(out)))
        return out

    def empty_hash(self):
        return self.hash(b"")


class Keccak256(Hash):
    kind = _lib.KECCAK256


class SM3(Hash):
    kind = _lib.SM3


def right160(h: bytes) -> bytes:
    """bcos::right160 (bcos-utilities/bcos-utilities/FixedBytes.h:666-671)."""
    return h[12:32]


class Merkle:
    """bcos::crypto::merkle::Merkle<Hasher, width> (Merkle.h:36); default width 2 (Merkle.h:36)."""

    def __init__(self, hasher: Hash, width: int = 2):
        if width < 2:
            raise ValueError("Width too short, at least 2")
        self.hasher, self.width = hasher, width

    def generate_merkle(self, origin_hashes):
        """generateMerkle (Merkle.h:170-208) -> the output vector as a list of 32-byte entries."""
        leaves = _u8(b"".join(bytes(h) for h in origin_hashes)).reshape(-1, 32)
        n = leaves.shape[0]
        if n == 0:
            raise ValueError("Empty input")
        ensure_device()
        size = int(lib().bcosgpu_merkle_size(n, self.width))
        levels = np.zeros((size, 32), dtype=np.uint8)
        root = np.zeros(32, dtype=np.uint8)
        check(lib().bcosgpu_merkle_root(self.hasher.kind, self.width, _lib.MERKLE_NEW, _ptr(leaves), n,
                                        _ptr(root), _ptr(levels)))
        return [levels[i].tobytes() for i in range(size)]

    def generate_merkle_bytes(self, origin_hashes):
        """generateMerkle into a std::vector<bytes> (BlockImpl's transactionsMerkle, BlockImpl.h:136;
        merkleBench.cpp:53-56): a list of entries, 4-byte count records and 32-byte nodes
        (bcosgpu_merkle_root with BCOSGPU_MERKLE_NEW_BYTES)."""
        leaves = _u8(b"".join(bytes(h) for h in origin_hashes)).reshape(-1, 32)
        n = leaves.shape[0]
        if n == 0:
            raise ValueError("Empty input")
        ensure_device()
        size = int(lib().bcosgpu_merkle_bytes_size(n, self.width))
        flat = np.zeros(size, dtype=np.uint8)
        root = np.zeros(32, dtype=np.uint8)
        check(lib().bcosgpu_merkle_root(self.hasher.kind, self.width, _lib.MERKLE_NEW_BYTES, _ptr(leaves), n,
                                        _ptr(root), _ptr(flat)))
        return split_merkle_bytes(flat.tobytes(), n)

    def root(self, leaves):
        """Root only (last element of generateMerkle's output); leaves: uint8[n,32] or list of bytes."""
        leaves = _u8(b"".join(bytes(h) for h in leaves) if isinstance(leaves, list) else leaves).reshape(-1, 32)
        n = leaves.shape[0]
        if n == 0:
            raise ValueError("Empty input")
        ensure_device()
        root = np.zeros(32, dtype=np.uint8)
        check(lib().bcosgpu_merkle_root(self.hasher.kind, self.width, _lib.MERKLE_NEW, _ptr(leaves), n,
                                        _ptr(root), None))
        return root.tobytes()

    def roots_batch(self, blocks):
        """Roots of many independent trees in one engine call (bcosgpu_merkle_roots_batch).
        blocks: list of uint8[n_b, 32] arrays (or lists of 32-byte strings).  An empty block yields
        the zero hash, as BlockImpl::calculateTransactionRoot does (BlockImpl.h:114-119)."""
        arrs = [_u8(b"".join(bytes(h) for h in b) if isinstance(b, list) else b).reshape(-1, 32) for b in blocks]
        nb = len(arrs)
        roots = np.zeros((max(nb, 1), 32), dtype=np.uint8)
        if nb == 0:
            return []
        off = np.zeros(nb + 1, dtype=np.uint64)
        off[1:] = np.cumsum([a.shape[0] for a in arrs], dtype=np.uint64)
        leaves = np.ascontiguousarray(np.concatenate(arrs, 0)) if off[-1] else np.zeros((1, 32), dtype=np.uint8)
        ensure_device()
        check(lib().bcosgpu_merkle_roots_batch(self.hasher.kind, self.width, _ptr(leaves), _ptr(off), nb, _ptr(roots)))
        return [roots[i].tobytes() for i in range(nb)]

    def generate_merkle_proofs(self, leaves, indices):
        """Batched generateMerkleProof(originHashes, merkle, index, out) (Merkle.h:121-168) on the GPU."""
        leaves = _u8(b"".join(bytes(h) for h in leaves) if isinstance(leaves, list) else leaves).reshape(-1, 32)
        n = leaves.shape[0]
        if n == 0:
            raise ValueError("Empty input")
        idx = np.ascontiguousarray(np.asarray(indices, dtype=np.uint64).reshape(-1))
        if idx.size and int(idx.max()) >= n:
            raise ValueError("Out of range!")
        m = idx.size
        ensure_device()
        stride = int(lib().bcosgpu_merkle_proof_stride(n, self.width))
        proofs = np.zeros((max(m, 1), stride, 32), dtype=np.uint8)
        plen = np.zeros(max(m, 1), dtype=np.uint32)
        if m:
            check(lib().bcosgpu_merkle_proofs(self.hasher.kind, self.width, _ptr(np.ascontiguousarray(leaves)), n, _ptr(idx),
                                              m, _ptr(proofs), _ptr(plen)))
        return [[proofs[q, e].tobytes() for e in range(int(plen[q]))] for q in range(m)]

    def generate_merkle_proof(self, origin_hashes, which):
        """generateMerkleProof: `which` is a leaf index, or a leaf hash (its first occurrence, Merkle.h:84-98)."""
        leaves = _u8(b"".join(bytes(h) for h in origin_hashes) if isinstance(origin_hashes, list)
                     else origin_hashes).reshape(-1, 32)
        if isinstance(which, (bytes, bytearray)):
            hits = np.nonzero((leaves == np.frombuffer(bytes(which), dtype=np.uint8)).all(axis=1))[0]
            if hits.size == 0:
                raise ValueError("Not found hash!")
            which = int(hits[0])
        return self.generate_merkle_proofs(leaves, [which])[0]

    def verify_merkle_proofs(self, proofs, hashes, roots):
        """Batched verifyMerkleProof (Merkle.h:45-81): list of proofs (lists of 32-byte entries), their leaf
        hashes, and one root per proof (or one shared root).  Returns bool[m]; an empty proof raises."""
        m = len(proofs)
        if any(len(p) == 0 for p in proofs):
            raise ValueError("Empty input proof!")
        if m == 0:
            return np.zeros(0, dtype=bool)
        stride = max(len(p) for p in proofs)
        buf = np.zeros((m, stride, 32), dtype=np.uint8)
        plen = np.array([len(p) for p in proofs], dtype=np.uint32)
        for q, p in enumerate(proofs):
            buf[q, :len(p)] = np.frombuffer(b"".join(bytes(e) for e in p), dtype=np.uint8).reshape(-1, 32)
        hs = _u8(b"".join(bytes(h) for h in hashes)).reshape(m, 32)
        rs = _u8(b"".join(bytes(r) for r in roots) if isinstance(roots, list) else bytes(roots)).reshape(-1, 32)
        ok = np.zeros(m, dtype=np.uint8)
        ensure_device()
        check(lib().bcosgpu_merkle_verify_proofs(self.hasher.kind, _ptr(buf), stride, _ptr(plen), _ptr(np.ascontiguousarray(hs)),
                                                 _ptr(np.ascontiguousarray(rs)), 1 if rs.shape[0] == m and m > 1 else 0, m,
                                                 _ptr(ok)))
        return ok == 1

    def verify_merkle_proof(self, proof, h, root):
        return bool(self.verify_merkle_proofs([proof], [bytes(h)], bytes(root))[0])


def split_merkle_bytes(flat: bytes, n: int):
    """The packed vector<bytes> layout -> its entries: each count record (4 bytes, big-endian) is
    followed by that many 32-byte nodes; n == 1 is the single 32-byte leaf."""
    if n == 1:
        return [flat[:32]]
    out, at = [], 0
    while at < len(flat):
        cnt = int.from_bytes(flat[at:at + 4], "big")
        out.append(flat[at:at + 4])
        at += 4
        for _ in range(cnt):
            out.append(flat[at:at + 32])
            at += 32
    return out


def calculate_merkle_proof_root(hasher: Hash, leaves) -> bytes:
    """protocol::calculateMerkleProofRoot (ParallelMerkleProof.cpp:32-69)."""
    leaves = _u8(b"".join(bytes(h) for h in leaves) if isinstance(leaves, list) else leaves).reshape(-1, 32)
    ensure_device()
    root = np.zeros(32, dtype=np.uint8)
    n = leaves.shape[0]
    d = leaves if n else np.zeros((1, 32), dtype=np.uint8)
    check(lib().bcosgpu_merkle_root(hasher.kind, 16, _lib.MERKLE_OLD, _ptr(d), n, _ptr(root), None))
    return root.tobytes()


class SignatureCrypto:
    """bcos::crypto::SignatureCrypto (Signature.h:31-59).  Single-item recover / verify go through the
    engine's explicit-device single calls (coalesced across threads, csrc/coalesce.hip); *_batch through
    the batch ABI.  An engine failure raises BcosGpuError, never InvalidSignature."""
    SIG_LEN = None
    SUITE = None

    def __init__(self, device=0):
        self.device = device

    def verify_batch(self, pubs, hashes, sigs):
        """Batched verify (bcosgpu_verify_batch): pubs uint8[n,64], hashes uint8[n,32],
        sigs uint8[n, stride >= 64] -> bool[n]  (sealer-signature checks, BlockValidator.cpp:141-182)."""
        pubs = _u8(pubs).reshape(-1, 64)
        n = pubs.shape[0]
        hashes = _u8(hashes).reshape(n, 32)
        sigs = _u8(sigs).reshape(n, -1) if n else np.zeros((0, 64), dtype=np.uint8)
        if sigs.shape[1] < 64:
            raise ValueError("signatures must hold at least r || s (64 bytes)")
        ok = np.zeros(n, dtype=np.uint8)
        if n:
            ensure_device(self.device)
            check(lib().bcosgpu_verify_batch(self.SUITE, _ptr(pubs), _ptr(hashes), _ptr(sigs), sigs.shape[1], n,
                                             _ptr(ok)))
        return ok.astype(bool)

    @staticmethod
    def _single(rc):
        if rc < 0:
            check(rc)
        return rc == 1


class Secp256k1Crypto(SignatureCrypto):
    """Secp256k1Crypto (Secp256k1Crypto.h:37-72); recover -> wedpr_secp256k1_recover_public_key."""
    SIG_LEN = 65
    SUITE = _lib.SUITE_SECP256K1

    def recover(self, hash32: bytes, sig: bytes) -> bytes:
        """Secp256k1Crypto::recover (Secp256k1Crypto.cpp:79-93): raises InvalidSignature."""
        h, s = bytes(hash32), bytes(sig)
        if len(h) != 32:
            raise ValueError("hash must be 32 bytes")
        pub = ctypes.create_string_buffer(64)
        if not self._single(lib().bcosgpu_secp256k1_recover(self.device, h, s, len(s), pub)):
            raise InvalidSignature("invalid signature: secp256k1Recover failed, msgHash : " + h.hex())
        return pub.raw

    def verify(self, pub: bytes, hash32: bytes, sig: bytes) -> bool:
        """secp256k1Verify (Secp256k1Crypto.cpp:51-63): libsecp256k1 verify, only sig[0:64] read."""
        p, h, s = bytes(pub), bytes(hash32), bytes(sig)
        if len(p) != 64 or len(h) != 32 or len(s) < 64:
            return False
        return self._single(lib().bcosgpu_secp256k1_verify(self.device, p, h, s, len(s)))

    def recover_batch(self, hashes, sigs, want_address=False):
        """hashes uint8[n,32]; sigs uint8[n,65] (or list of bytes; non-65-byte entries fail).
        Returns (pub uint8[n,64], ok bool[n]) or (pub, addr uint8[n,20], ok) with want_address."""
        hashes = _u8(hashes).reshape(-1, 32)
        n = hashes.shape[0]
        bad = np.zeros(n, dtype=bool)
        if isinstance(sigs, list):
            arr = np.zeros((n, 65), dtype=np.uint8)
            for i, s in enumerate(sigs):
                if len(s) == 65:
                    arr[i] = np.frombuffer(bytes(s), dtype=np.uint8)
                else:
                    bad[i] = True
                    arr[i, 64] = 0xFF  # any v > 3 fails
            sigs = arr
        sigs = _u8(sigs).reshape(n, 65)
        pub = np.zeros((n, 64), dtype=np.uint8)
        addr = np.zeros((n, 20), dtype=np.uint8)
        ok = np.zeros(n, dtype=np.uint8)
        if n:
            ensure_device(self.device)
            check(lib().bcosgpu_secp256k1_recover_batch(_ptr(hashes), _ptr(sigs), n, _ptr(pub),
                                                        _ptr(addr), _ptr(ok)))
        okb = ok.astype(bool) & ~bad
        return (pub, addr, okb) if want_address else (pub, okb)


class SM2Crypto(SignatureCrypto):
    """SM2Crypto / FastSM2Crypto: recover = verify against the embedded public key (SM2Crypto.cpp:81-92)."""
    SIG_LEN = 128
    SUITE = _lib.SUITE_SM2

    def verify(self, pub: bytes, hash32: bytes, sig: bytes) -> bool:
        """SM2Crypto::verify (SM2Crypto.cpp:66-79): r || s = sig[0:64], the given key."""
        p, h, s = bytes(pub), bytes(hash32), bytes(sig)
        if len(p) != 64 or len(h) != 32 or len(s) < 64:
            return False
        return self._single(lib().bcosgpu_sm2_verify(self.device, p, h, s[:64]))

    def recover(self, hash32: bytes, sig: bytes) -> bytes:
        """SM2Crypto::recover (SM2Crypto.cpp:81-92): sig = r || s || pub; raises InvalidSignature."""
        s = bytes(sig)
        if len(s) != 128 or not self.verify(s[64:], hash32, s[:64]):
            raise InvalidSignature("invalid signature: sm2 recover public key failed, msgHash : " + bytes(hash32).hex())
        return s[64:]

    def recover_batch(self, hashes, sigs, want_address=False):
        hashes = _u8(hashes).reshape(-1, 32)
        n = hashes.shape[0]
        bad = np.zeros(n, dtype=bool)
        if isinstance(sigs, list):
            arr = np.zeros((n, 128), dtype=np.uint8)
            for i, s in enumerate(sigs):
                if len(s) == 128:
                    arr[i] = np.frombuffer(bytes(s), dtype=np.uint8)
                else:
                    bad[i] = True  # SignatureDataWithPub: pub must be exactly 64 bytes
            sigs = arr
        sigs = _u8(sigs).reshape(n, 128)
        addr = np.zeros((n, 20), dtype=np.uint8)
        ok = np.zeros(n, dtype=np.uint8)
        if n:
            ensure_device(self.device)
            check(lib().bcosgpu_sm2_verify_batch(_ptr(hashes), _ptr(sigs), n, _ptr(addr), _ptr(ok)))
        okb = ok.astype(bool) & ~bad
        pub = sigs[:, 64:128].copy()
        return (pub, addr, okb) if want_address else (pub, okb)


class CryptoSuite:
    """bcos::crypto::CryptoSuite (CryptoSuite.h:33-67)."""

    def __init__(self, hash_impl: Hash, signature_impl: SignatureCrypto):
        self.hash_impl, self.signature_impl = hash_impl, signature_impl

    def hash(self, data: bytes) -> bytes:
        return self.hash_impl.hash(data)

    def calculate_address(self, pub: bytes) -> bytes:
        return right160(self.hash_impl.hash(pub))

    @property
    def suite(self):
        return _lib.SUITE_SM2 if isinstance(self.signature_impl, SM2Crypto) else _lib.SUITE_SECP256K1


def secp256k1_suite():
    """Keccak256 + Secp256k1Crypto (ProtocolInitializer.cpp:102-124, sm_crypto = false)."""
    return CryptoSuite(Keccak256(), Secp256k1Crypto())


def sm_suite():
    """SM3 + SM2 (ProtocolInitializer.cpp:102-124, sm_crypto = true)."""
    return CryptoSuite(SM3(), SM2Crypto())
