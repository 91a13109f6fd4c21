"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / timed CPU baseline.  See oracle/oracle.h for the reference citations.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
KECCAK256, SM3 = 0, 1
SUITE_SECP256K1, SUITE_SM2 = 0, 1

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        sigs = {
            "oracle_keccak256": (None, [P, S, P]), "oracle_sm3": (None, [P, S, P]),
            "oracle_hash": (None, [I, P, S, P]),
            "oracle_hash_batch": (None, [I, P, P, S, P, I]),
            "oracle_merkle": (I, [I, I, P, S, P, P, I]), "oracle_merkle_size": (S, [S, I]),
            "oracle_merkle_old": (None, [I, P, S, P]),
            "oracle_secp256k1_recover": (I, [P, P, S, P]), "oracle_secp256k1_pubkey": (I, [P, P]),
            "oracle_secp256k1_sign": (I, [P, P, P, P]), "oracle_secp256k1_verify": (I, [P, P, P, S]),
            "oracle_sm2_recover": (I, [P, P, S, P]), "oracle_sm2_pubkey": (I, [P, P]),
            "oracle_sm2_sign": (I, [P, P, P, P]), "oracle_sm2_za": (None, [P, P]),
            "oracle_tx_verify_batch": (None, [I, P, P, P, P, S, P, P, P, I]),
            "oracle_secp256k1_recover_batch": (None, [P, P, S, P, P, I]),
            "oracle_sm2_verify_batch": (None, [P, P, S, P, I]),
        }
        for k, (r, a) in sigs.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _b(x):
    return ctypes.c_char_p(bytes(x))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def keccak256(m: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_keccak256(_b(m), len(m), out)
    return out.raw


def sm3(m: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_sm3(_b(m), len(m), out)
    return out.raw


def hash_(hasher, m):
    return sm3(m) if hasher == SM3 else keccak256(m)


def hash_packed(hasher, data, offsets, nthreads=1):
    n = len(offsets) - 1
    out = np.zeros((n, 32), dtype=np.uint8)
    d = data if len(data) else np.zeros(1, dtype=np.uint8)
    lib().oracle_hash_batch(hasher, _p(d), _p(offsets), n, _p(out), nthreads)
    return out


def merkle(hasher, width, leaves, want_tree=False, nthreads=1):
    """leaves: uint8[n,32].  Returns root bytes (and the full output vector)."""
    leaves = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    n = leaves.shape[0]
    root = ctypes.create_string_buffer(32)
    size = 1 if n == 1 else lib().oracle_merkle_size(n, width)
    tree = np.zeros((max(size, 1), 32), dtype=np.uint8) if want_tree else None
    rc = lib().oracle_merkle(hasher, width, _p(leaves) if n else None, n, root,
                             _p(tree) if want_tree else None, nthreads)
    if rc:
        raise ValueError("Empty input")
    return (root.raw, tree) if want_tree else root.raw


def merkle_bytes_vector(hasher, width, leaves):
    """generateMerkle(originHashes, out) into a FRESH std::vector<bytes> -- BlockImpl's
    m_inner->transactionsMerkle (BlockImpl.h:136) and merkleBench's output (merkleBench.cpp:53-56):
    resizeTo(out, merkleNodes) appends empty buffers (Merkle.h:185-186, concepts/bcos-concepts/Basic.h:50-61),
    setNumberToHash's resizeTo(output, 4) makes each count record 4 bytes (Merkle.h:213-217), and
    hasher.final resizes each node to 32 (OpenSSLHasher.h:97-99); n == 1 is the single leaf
    (Merkle.h:177-182).  Pure Python over the C hashes: small inputs only."""
    leaves = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    n = leaves.shape[0]
    if n == 0:
        raise ValueError("Empty input")
    h = keccak256 if hasher == KECCAK256 else sm3
    if n == 1:
        return [leaves[0].tobytes()]
    out, level = [], [leaves[i].tobytes() for i in range(n)]
    while len(level) > 1:
        nxt = [h(b"".join(level[i:i + width])) for i in range(0, len(level), width)]
        out.append(len(nxt).to_bytes(4, "big"))
        out.extend(nxt)
        level = nxt
    return out


def merkle_old(hasher, leaves):
    leaves = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    root = ctypes.create_string_buffer(32)
    lib().oracle_merkle_old(hasher, _p(leaves) if leaves.shape[0] else None, leaves.shape[0], root)
    return root.raw


def secp256k1_recover(h, sig):
    pub = ctypes.create_string_buffer(64)
    rc = lib().oracle_secp256k1_recover(_b(h), _b(sig), len(sig), pub)
    return pub.raw if rc == 0 else None


def secp256k1_pubkey(sk):
    pub = ctypes.create_string_buffer(64)
    return pub.raw if lib().oracle_secp256k1_pubkey(_b(sk), pub) == 0 else None


def secp256k1_sign(sk, h, k):
    sig = ctypes.create_string_buffer(65)
    return sig.raw if lib().oracle_secp256k1_sign(_b(sk), _b(h), _b(k), sig) == 0 else None


def secp256k1_verify(pub, h, sig):
    return lib().oracle_secp256k1_verify(_b(pub), _b(h), _b(sig), len(sig)) == 0


def sm2_recover(h, sig):
    pub = ctypes.create_string_buffer(64)
    return pub.raw if lib().oracle_sm2_recover(_b(h), _b(sig), len(sig), pub) == 0 else None


def sm2_pubkey(sk):
    pub = ctypes.create_string_buffer(64)
    return pub.raw if lib().oracle_sm2_pubkey(_b(sk), pub) == 0 else None


def sm2_sign(sk, h, k):
    sig = ctypes.create_string_buffer(128)
    return sig.raw if lib().oracle_sm2_sign(_b(sk), _b(h), _b(k), sig) == 0 else None


def tx_verify_packed(suite, pre, pre_off, sig, sig_off, nthreads=1):
    n = len(pre_off) - 1
    txhash = np.zeros((n, 32), dtype=np.uint8)
    sender = np.zeros((n, 20), dtype=np.uint8)
    status = np.zeros(n, dtype=np.uint8)
    lib().oracle_tx_verify_batch(suite, _p(pre), _p(pre_off), _p(sig), _p(sig_off), n, _p(txhash),
                                 _p(sender), _p(status), nthreads)
    return txhash, sender, status


def secp256k1_recover_batch(hashes, sigs, nthreads=1):
    n = hashes.shape[0]
    pub = np.zeros((n, 64), dtype=np.uint8)
    ok = np.zeros(n, dtype=np.uint8)
    lib().oracle_secp256k1_recover_batch(_p(hashes), _p(sigs), n, _p(pub), _p(ok), nthreads)
    return pub, ok.astype(bool)


def sm2_verify_batch(hashes, sigs, nthreads=1):
    n = hashes.shape[0]
    ok = np.zeros(n, dtype=np.uint8)
    lib().oracle_sm2_verify_batch(_p(hashes), _p(sigs), n, _p(ok), nthreads)
    return ok.astype(bool)


def ecrecover(data: bytes):
    """EVM ecRecover precompile restated from bcos-executor/src/vm/Precompiled.cpp:443-482:
    rsv = r || s || (byte)(in[63] - 27); success -> 12 zero bytes || right160(keccak256(pub)),
    failure -> b"" (the precompile's empty output).  Input is read as 128 zero-padded bytes."""
    d = bytes(data)[:128].ljust(128, b"\0")
    rsv = d[64:128] + bytes([(d[63] - 27) & 0xFF])
    pub = secp256k1_recover(d[0:32], rsv)
    if pub is None:
        return b""
    return bytes(12) + keccak256(pub)[12:]


def receipt_preimage(version, gas_used, contract_address, status, output, logs, block_number):
    """impl_calculate<Hasher>(bcostars::TransactionReceipt) field order, restated from
    bcos-tars-protocol/bcos-tars-protocol/impl/TarsHashable.h:54-73: be32(version), gasUsed,
    contractAddress, be32(status), output, per log (address, topics..., data), be64(blockNumber).
    logs: list of (address: str, topics: list[bytes], data: bytes)."""
    out = bytearray()
    out += (version & 0xFFFFFFFF).to_bytes(4, "big")
    out += gas_used.encode()
    out += contract_address.encode()
    out += (status & 0xFFFFFFFF).to_bytes(4, "big")
    out += bytes(output)
    for address, topics, data in logs:
        out += address.encode()
        for t in topics:
            out += bytes(t)
        out += bytes(data)
    out += (block_number & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "big")
    return bytes(out)


def _count_record(c):
    return int(c).to_bytes(4, "big") + bytes(28)


def merkle_proof(hasher, width, leaves, index):
    """Merkle<H,width>::generateMerkleProof(originHashes, merkle, index, out), restated from
    bcos-crypto/bcos-crypto/merkle/Merkle.h:121-168 over this oracle's tree (list of 32-byte entries)."""
    leaves = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    n = leaves.shape[0]
    if index >= n:
        raise ValueError("Out of range!")
    _, tree = merkle(hasher, width, leaves, want_tree=True)
    if n == 1:
        return [tree[0].tobytes()]
    index -= (index + width) % width  # indexAlign (Merkle.h:211)
    count = min(n - index, width)
    out = [_count_record(count)] + [leaves[j].tobytes() for j in range(index, index + count)]
    pos = 0
    while pos < tree.shape[0]:
        index //= width
        index -= (index + width) % width
        level_len = int.from_bytes(tree[pos, :4].tobytes(), "big")
        pos += 1
        if level_len == 1:
            break
        nxt = min(level_len - index, width)
        out.append(_count_record(nxt))
        out += [tree[pos + j].tobytes() for j in range(index, index + nxt)]
        pos += level_len
    return out


def merkle_verify_proof(hasher, proof, h, root):
    """verifyMerkleProof (Merkle.h:45-81); empty proof raises like std::invalid_argument."""
    if len(proof) == 0:
        raise ValueError("Empty input proof!")
    h = bytes(h)
    if len(proof) > 1:
        it = 0
        while it < len(proof):
            count = int.from_bytes(proof[it][:4], "big")
            it += 1
            group = proof[it:it + count]
            if len(group) < count or h not in group:
                return False
            h = hash_(hasher, b"".join(group))
            it += count
    return h == bytes(root)


def tx_preimage(version, chain_id, group_id, block_limit, nonce, to, input_, abi):
    """impl_calculate<Hasher>(bcostars::Transaction) field order, restated from
    bcos-tars-protocol/bcos-tars-protocol/impl/TarsHashable.h:29-40."""
    return ((version & 0xFFFFFFFF).to_bytes(4, "big") + chain_id.encode() + group_id.encode()
            + (block_limit & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "big") + nonce.encode() + to.encode() + bytes(input_)
            + abi.encode())


# ---------------------------------------------------------------- OpenSSL stand-in (CPU baseline)
STANDIN = os.path.join(HERE, "libstandin.so")
_standin = None


def standin():
    """oracle/libstandin.so (standin_openssl.c): the reference's per-tx path over OpenSSL 1.1.1's
    libcrypto EC, the declared CPU stand-in of BASELINE.md §3.  None when it is not built (no
    OpenSSL headers) or its libcrypto does not load."""
    global _standin
    if _standin is None:
        if not os.path.exists(STANDIN):
            subprocess.run(["make", "-s", "-C", HERE, "standin"], check=False)
        try:
            L = ctypes.CDLL(STANDIN)
        except OSError:
            return None
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.standin_version.restype = ctypes.c_char_p
        L.standin_version.argtypes = []
        L.standin_tx_verify_batch.restype = None
        L.standin_tx_verify_batch.argtypes = [I, P, P, P, P, S, P, P, P, I]
        L.standin_hash.restype = I
        L.standin_hash.argtypes = [I, P, S, P]
        L.standin_merkle_root.restype = I
        L.standin_merkle_root.argtypes = [I, I, P, S, P, I]
        L.standin_verify_batch.restype = None
        L.standin_verify_batch.argtypes = [I, P, P, P, S, S, P, I]
        _standin = L
    return _standin


def standin_version():
    L = standin()
    return L.standin_version().decode() if L else None


def standin_tx_verify_packed(suite, pre, pre_off, sig, sig_off, nthreads=1):
    n = len(pre_off) - 1
    txhash = np.zeros((n, 32), dtype=np.uint8)
    sender = np.zeros((n, 20), dtype=np.uint8)
    status = np.zeros(n, dtype=np.uint8)
    standin().standin_tx_verify_batch(suite, _p(pre), _p(pre_off), _p(sig), _p(sig_off), n, _p(txhash),
                                      _p(sender), _p(status), nthreads)
    return txhash, sender, status


def standin_verify_batch(suite, pubs, hashes, sigs, nthreads=1):
    """SignatureCrypto::verify with known keys over OpenSSL (secp256k1: libsecp256k1 verify semantics,
    low-S; SM2: EVP with the default ID).  pubs [n,64], hashes [n,32], sigs [n, stride >= 64]."""
    pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1, 64)
    n = pubs.shape[0]
    hashes = np.ascontiguousarray(hashes, dtype=np.uint8).reshape(n, 32)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(n, -1)
    ok = np.zeros(n, dtype=np.uint8)
    standin().standin_verify_batch(suite, _p(pubs), _p(hashes), _p(sigs), sigs.shape[1], n, _p(ok), nthreads)
    return ok.astype(bool)


def standin_hash(hasher, data):
    """OpenSSLHasher<SM3 | Keccak256> (OpenSSLHasher.h:22-143) over OpenSSL 1.1.1's EVP (stand-in build)."""
    out = np.zeros(32, dtype=np.uint8)
    d = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    if standin().standin_hash(hasher, _p(d), len(data), _p(out)) != 0:
        raise RuntimeError("OpenSSL hasher failed (KECCAK1600_CTX layout?)")
    return out.tobytes()


def standin_merkle_root(hasher, width, leaves, nthreads=1):
    """Merkle<H, width>::generateMerkle's root (Merkle.h:170-261) with the reference's OpenSSL hashers,
    levels parallel over nthreads (the reference CPU path merkleBench.cpp times)."""
    leaves = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    root = np.zeros(32, dtype=np.uint8)
    if standin().standin_merkle_root(hasher, width, _p(leaves), leaves.shape[0], _p(root), nthreads) != 0:
        raise RuntimeError("standin_merkle_root failed")
    return root.tobytes()
