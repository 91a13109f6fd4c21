"""The C-ABI library builds for gfx950, loads, and exports every symbol include/bcos_gpu.h declares
(CPU; no compute calls).  Also checks host-side logic that needs no GPU."""
import ctypes
import subprocess

import bcos_gpu
from bcos_gpu import _lib


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib._SIGS) == set(syms), set(_lib._SIGS) ^ set(syms)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          "--input=" + _lib.LIB_PATH], capture_output=True, text=True)
    if out.returncode == 0 and out.stdout:
        assert "gfx950" in out.stdout
    else:  # fall back to scanning the fat binary for the target id
        with open(_lib.LIB_PATH, "rb") as f:
            assert b"gfx950" in f.read()


def test_cheap_calls_without_gpu():
    L = _lib.lib()
    assert L.bcosgpu_version() == 1
    assert L.bcosgpu_merkle_size(100000, 16) == 6250 + 391 + 25 + 2 + 1 + 5
    assert L.bcosgpu_merkle_size(1, 2) == 1
    assert L.bcosgpu_merkle_size(3, 2) == 2 + 1 + 2


def test_tx_preimage_layout():
    """TarsHashable.h:29-40: be32(version) || chainID || groupID || be64(blockLimit) || nonce || to || input || abi"""
    t = bcos_gpu.TransactionData(version=1, chain_id="chain0", group_id="group0", block_limit=500,
                                 nonce="123", to="ab" * 20, input=b"\x01\x02", abi="")
    p = t.preimage()
    assert p[:4] == b"\x00\x00\x00\x01" and p[4:16] == b"chain0group0"
    assert p[16:24] == (500).to_bytes(8, "big") and p[24:27] == b"123"
    assert p[27:67] == b"ab" * 20 and p[67:] == b"\x01\x02"
