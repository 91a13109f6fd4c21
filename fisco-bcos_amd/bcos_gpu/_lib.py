"""ctypes binding of libbcosgpu.so (include/bcos_gpu.h).

The product path is the HIP library: if it is missing or cannot be loaded this module raises --
there is no CPU fallback anywhere in the package.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libbcosgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "bcos_gpu.h")

OK, E_ARG, E_HIP, E_NODEV, E_EMPTY = 0, -1, -2, -3, -4
WEDPR_ENGINE_ERROR = -2
KECCAK256, SM3 = 0, 1
SUITE_SECP256K1, SUITE_SM2 = 0, 1
MERKLE_NEW, MERKLE_OLD, MERKLE_NEW_BYTES = 0, 1, 2


class BcosGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"bcosgpu error {code}: {msg}")
        self.code = code


_lib = None

_P = ctypes.c_void_p
_U8P = ctypes.c_char_p
_SZ = ctypes.c_size_t
_I = ctypes.c_int

_SIGS = {
    "bcosgpu_version": (_I, []),
    "bcosgpu_device_count": (_I, []),
    "bcosgpu_init": (_I, [_I]),
    "bcosgpu_init_ex": (_I, [_I, _I]),
    "bcosgpu_set_tx_kernel_policy": (_I, [_I, _I, _I, _I]),
    "bcosgpu_last_error": (ctypes.c_char_p, []),
    "bcosgpu_merkle_size": (ctypes.c_uint64, [ctypes.c_uint64, _I]),
    "bcosgpu_hash_batch": (_I, [_I, _P, _P, _SZ, _P]),
    "bcosgpu_keccak256_batch": (_I, [_P, _P, _SZ, _P]),
    "bcosgpu_sm3_batch": (_I, [_P, _P, _SZ, _P]),
    "bcosgpu_hash_batch_dev": (_I, [_I, _P, _P, _SZ, _P, _P]),
    "bcosgpu_merkle_root": (_I, [_I, _I, _I, _P, _SZ, _P, _P]),
    "bcosgpu_merkle_root_dev": (_I, [_I, _I, _P, _SZ, _P, _P, _P]),
    "bcosgpu_merkle_bytes_size": (ctypes.c_uint64, [ctypes.c_uint64, _I]),
    "bcosgpu_merkle_tree_bytes_dev": (_I, [_I, _P, _SZ, _P, _P]),
    "bcosgpu_merkle_frontier_dev": (_I, [_I, _I, _P, _SZ, _I, _P, _P, _P]),
    "bcosgpu_merkle_roots_work_size": (ctypes.c_uint64, [ctypes.c_uint64, _SZ, _I]),
    "bcosgpu_merkle_roots_batch": (_I, [_I, _I, _P, _P, _SZ, _P]),
    "bcosgpu_merkle_roots_batch_dev": (_I, [_I, _I, _P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_merkle_proof_stride": (ctypes.c_uint64, [ctypes.c_uint64, _I]),
    "bcosgpu_merkle_proofs": (_I, [_I, _I, _P, _SZ, _P, _SZ, _P, _P]),
    "bcosgpu_merkle_proofs_dev": (_I, [_I, _P, _SZ, _P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_merkle_verify_proofs": (_I, [_I, _P, ctypes.c_uint64, _P, _P, _P, _I, _SZ, _P]),
    "bcosgpu_merkle_verify_proofs_dev": (_I, [_I, _P, ctypes.c_uint64, _P, _P, _P, _I, _SZ, _P, _P]),
    "bcosgpu_secp256k1_recover_batch": (_I, [_P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_secp256k1_recover_batch_dev": (_I, [_P, _P, _SZ, _P, _P, _P, _P]),
    "bcosgpu_sm2_verify_batch": (_I, [_P, _P, _SZ, _P, _P]),
    "bcosgpu_sm2_verify_batch_dev": (_I, [_P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_secp256k1_sign_batch_dev": (_I, [_P, _P, _SZ, _P, _P, _P, _P]),
    "bcosgpu_sm2_sign_batch_dev": (_I, [_P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_verify_batch": (_I, [_I, _P, _P, _P, _SZ, _SZ, _P]),
    "bcosgpu_verify_batch_dev": (_I, [_I, _P, _P, _P, _SZ, _SZ, _P, _P]),
    "bcosgpu_register_keys": (_I, [_I, _I, _P, _SZ, _P]),
    "bcosgpu_verify_keyed_batch_dev": (_I, [_I, _P, _P, _P, _SZ, _SZ, _P, _P]),
    "bcosgpu_key_cache_info": (_I, [_I, _I, _P]),
    "bcosgpu_clear_keys": (_I, [_I, _I]),
    "bcosgpu_ecrecover_batch": (_I, [_P, _SZ, _P, _P]),
    "bcosgpu_ecrecover_batch_dev": (_I, [_P, _SZ, _P, _P, _P]),
    "bcosgpu_tx_verify_batch": (_I, [_I, _P, _P, _P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_tx_verify_batch_dev": (_I, [_I, _P, _P, _P, _P, _SZ, _P, _P, _P, _P]),
    "bcosgpu_tx_preimage_size": (ctypes.c_uint64, [_P, _SZ]),
    "bcosgpu_pack_tx_preimages": (_I, [_P, _SZ, _P, ctypes.c_uint64, _P]),
    "bcosgpu_receipt_preimage_size": (ctypes.c_uint64, [_P, _SZ]),
    "bcosgpu_pack_receipt_preimages": (_I, [_P, _SZ, _P, ctypes.c_uint64, _P]),
    "bcosgpu_apply_receipt_data_hashes": (None, [_P, _SZ, _P]),
    "bcosgpu_receipt_roots": (_I, [_I, _P, _P, _SZ, _P, _P]),
    "bcosgpu_tars_decode_work_size": (ctypes.c_uint64, [_SZ]),
    "bcosgpu_tars_tx_decode_dev": (_I, [_P, _P, _SZ, _P, _P, _P, _P, _P, _P, ctypes.c_uint64, _P]),
    "bcosgpu_tars_tx_verify_batch": (_I, [_I, _P, _P, _SZ, _I, _I, _P, _P, _P]),
    "bcosgpu_tars_tx_verify_batch_dev": (_I, [_I, _P, _P, _SZ, _I, _I, _P, _P, _P, _P, _P, ctypes.c_uint64, _P, _P,
                                              _P, _P]),
    "bcosgpu_secp256k1_recover": (_I, [_I, _P, _P, _SZ, _P]),
    "bcosgpu_secp256k1_verify": (_I, [_I, _P, _P, _P, _SZ]),
    "bcosgpu_sm2_verify": (_I, [_I, _P, _P, _P]),
    "bcosgpu_coalesce_stats": (_I, [_I, _P, _I]),
    "bcosgpu_init_devices": (_I, [_P, _I]),
    "bcosgpu_secp256k1_recover_batch_multi": (_I, [_P, _I, _P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_sm2_verify_batch_multi": (_I, [_P, _I, _P, _P, _SZ, _P, _P]),
    "bcosgpu_verify_batch_multi": (_I, [_P, _I, _I, _P, _P, _P, _SZ, _SZ, _P]),
    "bcosgpu_tx_verify_batch_multi": (_I, [_P, _I, _I, _P, _P, _P, _P, _SZ, _P, _P, _P]),
    "bcosgpu_block_verify_multi": (_I, [_P, _I, _I, _P, _P, _P, _P, _SZ, _I, _P, _P, _P, _P]),
    "bcosgpu_merkle_root_multi": (_I, [_P, _I, _I, _I, _P, _SZ, _P]),
    "bcosgpu_blocks_verify_multi": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _SZ, _I, _P, _P, _P, _P]),
    "bcosgpu_wedpr_secp256k1_recover_public_key": (ctypes.c_int8, [_P, _P, _P]),
    "bcosgpu_wedpr_sm2_verify": (ctypes.c_int8, [_P, _P, _P]),
    "bcosgpu_wedpr_secp256k1_verify": (ctypes.c_int8, [_P, _P, _P]),
}


def header_symbols():
    """Every function declared in include/bcos_gpu.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(bcosgpu_\w+)\s*\(", text)))


def lib():
    """Load libbcosgpu.so (raises OSError when the HIP build is missing)."""
    global _lib
    if _lib is None:
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so, soname libamdhip64.so.7); load
        # it first so libbcosgpu.so binds to that same runtime instead of a second copy from
        # /opt/rocm -- two HIP runtimes in one process cannot share devices, pointers or streams.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `make -C fisco-bcos_amd` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise BcosGpuError(rc, lib().bcosgpu_last_error().decode(errors="replace"))
    return rc


_inited = set()


def ensure_device(device=0):
    """Initialise the engine on `device` (fails loudly without a gfx950 GPU)."""
    if device not in _inited:
        check(lib().bcosgpu_init(device))
        _inited.add(device)


def set_tx_kernel_policy(split=-1, occupancy=0, coop=2, field=1):
    """bcosgpu_set_tx_kernel_policy: force a tx-verify kernel variant (tests / tuning); the defaults
    restore the size-based choice (field 1: the 10 x 26-bit secp256k1 point arithmetic)."""
    check(lib().bcosgpu_set_tx_kernel_policy(split, occupancy, coop, field))


def register_keys(suite, pubs, device=0):
    """bcosgpu_register_keys: comb tables for the keys pubs uint8[n, 64] (the sealer set) on `device`.
    Returns the int32 slot of each key (-1 where the cache is full)."""
    import numpy as np
    ensure_device(device)
    p = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1, 64)
    slots = np.full(p.shape[0], -1, dtype=np.int32)
    if p.shape[0]:
        rc = lib().bcosgpu_register_keys(device, suite, p.ctypes.data, p.shape[0], slots.ctypes.data)
        if rc < 0:
            check(rc)
    return slots


def key_cache_info(suite, device=0):
    """{keys, capacity, keyed (signatures verified on the registered-key kernel), generic, built}."""
    import numpy as np
    out = np.zeros(5, dtype=np.int64)
    check(lib().bcosgpu_key_cache_info(device, suite, out.ctypes.data))
    return dict(zip(("keys", "capacity", "keyed", "generic", "built"), (int(x) for x in out)))


def clear_keys(suite, device=0):
    check(lib().bcosgpu_clear_keys(device, suite))
