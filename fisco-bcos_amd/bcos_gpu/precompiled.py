"""EVM ecRecover precompile, batched on the GPU.

  ecRecover(bytesConstRef _in)   bcos-executor/src/vm/Precompiled.cpp:443-482
    _in = hash(32) || v(32) || r(32) || s(32); rsv = r || s || (byte)(_in[63] - 27);
    wedpr_secp256k1_recover_public_key -> {true, 12 zero bytes || right160(keccak256(pub))};
    on failure {true, {}} (an empty output).
"""
import numpy as np

from ._lib import check, ensure_device, lib
from .crypto import _ptr, _u8


def ec_recover_batch(inputs):
    """inputs: list of bytes (each zero-padded / truncated to 128 bytes, as the EVM call data the
    precompile reads) or uint8[n,128] -> (out uint8[n,32], ok bool[n])."""
    if isinstance(inputs, list):
        arr = np.zeros((len(inputs), 128), dtype=np.uint8)
        for i, m in enumerate(inputs):
            m = bytes(m)[:128]
            arr[i, :len(m)] = np.frombuffer(m, dtype=np.uint8)
        inputs = arr
    inputs = np.ascontiguousarray(_u8(inputs).reshape(-1, 128))
    n = inputs.shape[0]
    out = np.zeros((n, 32), dtype=np.uint8)
    ok = np.zeros(n, dtype=np.uint8)
    if n:
        ensure_device()
        check(lib().bcosgpu_ecrecover_batch(_ptr(inputs), n, _ptr(out), _ptr(ok)))
    return out, ok.astype(bool)


def ec_recover(data: bytes):
    """Single call with the reference's return shape: (True, 32-byte output) or (True, b"")."""
    out, ok = ec_recover_batch([data])
    return True, (out[0].tobytes() if ok[0] else b"")
