"""Device-resident entry points over torch tensors (HBM-resident inputs, stream-ordered launches).

PyTorch only provides the device memory and the stream here; the compute is libbcosgpu.so.
Every function takes uint8 / int64 CUDA tensors and launches on torch's current stream (or the
given one) without synchronising.
"""
import torch

from . import _lib
from ._lib import check, ensure_device, lib

KECCAK256, SM3 = _lib.KECCAK256, _lib.SM3
SUITE_SECP256K1, SUITE_SM2 = _lib.SUITE_SECP256K1, _lib.SUITE_SM2


def _s(stream):
    return (stream if stream is not None else torch.cuda.current_stream()).cuda_stream


def _p(t):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "device tensors must be contiguous CUDA tensors"
    return t.data_ptr()


def _dev(t):
    ensure_device(t.device.index if t.device.index is not None else 0)


def hash_batch(hasher, data, offsets, out, stream=None):
    """data uint8[B], offsets int64[n+1], out uint8[n,32]."""
    _dev(out)
    n = offsets.numel() - 1
    check(lib().bcosgpu_hash_batch_dev(hasher, _p(data), _p(offsets), n, _p(out), _s(stream)))


def merkle_size(n, width):
    return int(lib().bcosgpu_merkle_size(n, width))


def merkle_root(hasher, width, leaves, tree, root, stream=None):
    """leaves uint8[n,32]; tree uint8[merkle_size(n,width),32]; root uint8[32]."""
    _dev(leaves)
    check(lib().bcosgpu_merkle_root_dev(hasher, width, _p(leaves), leaves.shape[0], _p(tree), _p(root),
                                        _s(stream)))


def merkle_frontier(hasher, width, leaves, levels, work, frontier, stream=None):
    """Reference-tree level `levels` over a width^levels-aligned shard (bcosgpu_merkle_frontier_dev)."""
    _dev(leaves)
    check(lib().bcosgpu_merkle_frontier_dev(hasher, width, _p(leaves), leaves.shape[0], levels, _p(work),
                                            _p(frontier), _s(stream)))


def merkle_roots_work_size(total_leaves, nblocks, width):
    return int(lib().bcosgpu_merkle_roots_work_size(total_leaves, nblocks, width))


def merkle_roots_batch(hasher, width, leaves, block_off, work, roots, stream=None):
    """Roots of many blocks' trees (bcosgpu_merkle_roots_batch_dev).  leaves uint8[N,32] (device),
    block_off: host uint64 numpy array [nblocks+1] of row indices into `leaves`, work: uint8 device
    tensor >= merkle_roots_work_size bytes, roots uint8[nblocks,32]."""
    import ctypes
    import numpy as np
    _dev(leaves)
    bo = np.ascontiguousarray(block_off, dtype=np.uint64)
    nb = bo.size - 1
    base = leaves[int(bo[0]):] if nb > 0 and int(bo[0]) < leaves.shape[0] else leaves
    check(lib().bcosgpu_merkle_roots_batch_dev(hasher, width, _p(base), bo.ctypes.data_as(ctypes.c_void_p), nb,
                                               _p(work), _p(roots), _s(stream)))


def verify_keyed(suite, slots, hashes, sigs, ok, stream=None):
    """SignatureCrypto::verify against registered keys (bcosgpu_verify_keyed_batch_dev): slots int32[n]
    (from _lib.register_keys), hashes uint8[n,32], sigs uint8[n, stride >= 64] (r || s read) -> ok uint8[n]."""
    _dev(ok)
    n = slots.numel()
    check(lib().bcosgpu_verify_keyed_batch_dev(suite, _p(slots), _p(hashes), _p(sigs), sigs.shape[1] if n else 64, n,
                                               _p(ok), _s(stream)))


def secp256k1_recover(hashes, sigs, pub, addr, ok, stream=None):
    """hashes uint8[n,32], sigs uint8[n,65] -> pub uint8[n,64] (or None), addr uint8[n,20] (or None), ok uint8[n]."""
    _dev(hashes)
    check(lib().bcosgpu_secp256k1_recover_batch_dev(_p(hashes), _p(sigs), hashes.shape[0], _p(pub), _p(addr),
                                                    _p(ok), _s(stream)))


def sm2_verify(hashes, sigs, addr, ok, stream=None):
    """hashes uint8[n,32], sigs uint8[n,128] (r||s||pub) -> addr uint8[n,20] (or None), ok uint8[n]."""
    _dev(hashes)
    check(lib().bcosgpu_sm2_verify_batch_dev(_p(hashes), _p(sigs), hashes.shape[0], _p(addr), _p(ok), _s(stream)))


def secp256k1_sign(sks, hashes, pub, sigs, ok, stream=None):
    _dev(sks)
    check(lib().bcosgpu_secp256k1_sign_batch_dev(_p(sks), _p(hashes), sks.shape[0], _p(pub), _p(sigs), _p(ok),
                                                 _s(stream)))


def sm2_sign(sks, hashes, sigs, ok, stream=None):
    _dev(sks)
    check(lib().bcosgpu_sm2_sign_batch_dev(_p(sks), _p(hashes), sks.shape[0], _p(sigs), _p(ok), _s(stream)))


def tx_verify(suite, pre, pre_off, sig, sig_off, txhash, sender, status, stream=None):
    """Batched Transaction::verify; all device tensors (see bcosgpu_tx_verify_batch_dev)."""
    _dev(pre)
    n = pre_off.numel() - 1
    check(lib().bcosgpu_tx_verify_batch_dev(suite, _p(pre), _p(pre_off), _p(sig), _p(sig_off), n, _p(txhash),
                                            _p(sender), _p(status), _s(stream)))


def tars_decode_work_size(n):
    return int(lib().bcosgpu_tars_decode_work_size(n))


def tars_tx_decode(enc, enc_off, pre, pre_off, sig, sig_off, dec_status, work, stream=None):
    """Device Tars decode of n transactions into the packed preimage / signature layout
    (bcosgpu_tars_tx_decode_dev); dec_status may be None."""
    _dev(enc)
    n = enc_off.numel() - 1
    check(lib().bcosgpu_tars_tx_decode_dev(_p(enc), _p(enc_off), n, _p(pre), _p(pre_off), _p(sig), _p(sig_off),
                                           None if dec_status is None else _p(dec_status), _p(work),
                                           work.numel() * work.element_size(), _s(stream)))


def tars_tx_verify(suite, enc, enc_off, pre, pre_off, sig, sig_off, work, txhash, sender, status, check_sig=True,
                   check_hash=False, stream=None):
    """Device createTransaction: decode + hash (+ Transaction::verify when check_sig)
    (bcosgpu_tars_tx_verify_batch_dev)."""
    _dev(enc)
    n = enc_off.numel() - 1
    check(lib().bcosgpu_tars_tx_verify_batch_dev(suite, _p(enc), _p(enc_off), n, int(bool(check_sig)),
                                                 int(bool(check_hash)), _p(pre),
                                                 _p(pre_off), _p(sig), _p(sig_off), _p(work),
                                                 work.numel() * work.element_size(), _p(txhash), _p(sender),
                                                 _p(status), _s(stream)))
