"""Synthetic signed-transaction batches, built on the device.

Preimages follow TarsHashable.h:16-41 with the survey's synthetic field values: version 0,
chainID "chain0", groupID "group0", blockLimit 500, nonce = 19-digit decimal counter, to = 40 hex
chars of random bytes, input = 68 random bytes, abi "" -> 151-byte preimages (2 Keccak blocks).
One distinct key per tx; signatures come from the engine's own signing kernels
(bcosgpu_*_sign_batch_dev, deterministic nonces), then a fraction is corrupted:
  secp256k1: `flip_frac` get one bit of s flipped (still recovers, to a different sender -- the
             reference accepts those, TxPoolTest.cpp:469-489); `bad_v_frac` get v = 4 (must fail).
  SM2:       `flip_frac` get one bit flipped (must fail).
"""
import numpy as np
import torch

from . import device

PREIMAGE_LEN = 151
N_SECP = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
N_SM2 = 0xFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123


def preimages(n, seed=0xF15C0BC5):
    """uint8[n, 151] preimages of synthetic TransactionData (TarsHashable.h:29-40 field order)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, PREIMAGE_LEN), dtype=np.uint8)
    out[:, 0:4] = 0  # be32(version = 0)
    out[:, 4:10] = np.frombuffer(b"chain0", dtype=np.uint8)
    out[:, 10:16] = np.frombuffer(b"group0", dtype=np.uint8)
    out[:, 16:24] = np.frombuffer((500).to_bytes(8, "big"), dtype=np.uint8)
    nonce = np.uint64(10 ** 18) + np.arange(n, dtype=np.uint64) + np.uint64(seed & 0xFFFFFFFF)
    for d in range(18, -1, -1):  # 19 decimal digits, most significant first
        out[:, 24 + d] = (nonce % np.uint64(10)).astype(np.uint8) + ord("0")
        nonce //= np.uint64(10)
    to = rng.integers(0, 256, size=(n, 20), dtype=np.uint8)
    hexd = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
    out[:, 43:83:2] = hexd[to >> 4]
    out[:, 44:84:2] = hexd[to & 15]
    out[:, 83:151] = rng.integers(0, 256, size=(n, 68), dtype=np.uint8)
    return out


def secret_keys(n, seed, order):
    """uint8[n, 32] big-endian secret keys, uniformly random in [1, order - 2]."""
    rng = np.random.default_rng(seed ^ 0x5EC)
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x7F  # < 2^255 < order - 2 for both curves
    sk[:, 31] |= 1  # never zero
    return sk


class SignedBatch:
    """Device-resident batch: preimages, offsets, signatures (+ offsets), ground-truth metadata."""

    def __init__(self, suite, pre, pre_off, sig, sig_off, sig_len, corrupted, n):
        self.suite, self.pre, self.pre_off, self.sig, self.sig_off = suite, pre, pre_off, sig, sig_off
        self.sig_len, self.corrupted, self.n = sig_len, corrupted, n


def make_batch(suite, n, seed=0xF15C0BC5, flip_frac=0.01, bad_v_frac=0.001, dev="cuda"):
    """Build n signed synthetic transactions on `dev` for suite 0 (secp256k1) or 1 (SM2)."""
    pre_h = preimages(n, seed)
    pre = torch.from_numpy(pre_h.reshape(-1)).to(dev)
    pre_off = torch.arange(0, (n + 1) * PREIMAGE_LEN, PREIMAGE_LEN, dtype=torch.int64, device=dev)
    hasher = device.SM3 if suite == device.SUITE_SM2 else device.KECCAK256
    txhash = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    device.hash_batch(hasher, pre, pre_off, txhash)
    sk = torch.from_numpy(secret_keys(n, seed, N_SM2 if suite else N_SECP)).to(dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    if suite == device.SUITE_SM2:
        sig_len = 128
        sig = torch.empty((n, 128), dtype=torch.uint8, device=dev)
        device.sm2_sign(sk, txhash, sig, ok)
    else:
        sig_len = 65
        sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
        pub = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        device.secp256k1_sign(sk, txhash, pub, sig, ok)
    torch.cuda.synchronize()
    if not bool(ok.all()):
        raise RuntimeError("synthetic signing produced a degenerate signature")
    rng = np.random.default_rng(seed ^ 0xBAD)
    corrupted = np.zeros(n, dtype=np.uint8)  # 1 = bit flip, 2 = bad v
    flips = rng.random(n) < flip_frac
    idx = np.nonzero(flips)[0]
    if len(idx):
        byte = rng.integers(32, 64, size=len(idx)) if suite != device.SUITE_SM2 else rng.integers(0, 64, size=len(idx))
        bit = rng.integers(0, 8, size=len(idx))
        flat = sig.view(-1)
        pos = torch.from_numpy(idx * sig_len + byte).to(dev)
        mask = torch.from_numpy((1 << bit).astype(np.uint8)).to(dev)
        flat[pos] ^= mask
        corrupted[idx] = 1
    if suite != device.SUITE_SM2 and bad_v_frac > 0:
        badv = np.nonzero((rng.random(n) < bad_v_frac) & ~flips)[0]
        if len(badv):
            sig[torch.from_numpy(badv).to(dev), 64] = 4
            corrupted[badv] = 2
    sig_off = torch.arange(0, (n + 1) * sig_len, sig_len, dtype=torch.int64, device=dev)
    return SignedBatch(suite, pre, pre_off, sig.view(-1), sig_off, sig_len, corrupted, n)


def tars_encodings(b: SignedBatch):
    """The batch as Tars-encoded bcostars::Transaction bytes (TransactionImpl::encode), built on the
    device from the fixed-layout preimages: data {chainID, groupID, blockLimit 500, nonce, to, input},
    dataHash (the tx hash) and signature, in the exact bytes bcos_gpu.tars.encode_transaction writes.
    Returns (uint8 enc[n * L], int64 offsets[n + 1])."""
    n, dev = b.n, b.pre.device
    pre = b.pre.view(n, PREIMAGE_LEN)
    txhash = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    device.hash_batch(device.SM3 if b.suite == device.SUITE_SM2 else device.KECCAK256, b.pre, b.pre_off, txhash)

    def const(bs):
        return torch.tensor(list(bs), dtype=torch.uint8, device=dev).expand(n, len(bs))

    sig_head = b"\x3d\x00\x01\x00\x80" if b.sig_len == 128 else b"\x3d\x00\x00" + bytes([b.sig_len])
    cols = [const(b"\x1a\x26\x06"), pre[:, 4:10], const(b"\x36\x06"), pre[:, 10:16],
            const(b"\x41\x01\xf4\x56\x13"), pre[:, 24:43], const(b"\x66\x28"), pre[:, 43:83],
            const(b"\x7d\x00\x00\x44"), pre[:, 83:151], const(b"\x0b\x2d\x00\x00\x20"), txhash,
            const(sig_head), b.sig.view(n, b.sig_len)]
    enc = torch.cat(cols, dim=1).contiguous()
    L = enc.shape[1]
    off = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
    return enc.view(-1), off
