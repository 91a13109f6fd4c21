"""The C-ABI library builds for gfx950, loads, and exports every symbol include/bcos_gpu.h declares
(CPU; no compute calls).  Also checks host-side logic that needs no GPU."""
import ctypes
import subprocess

import numpy as np

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


def test_library_binds_no_hip_symbol_newer_than_torchs_runtime():
    """libbcosgpu.so is loaded into processes that already hold torch's HIP runtime (torch/lib/libamdhip64.so,
    ROCm 7.0 -- _lib.lib() imports torch first so both share it); a HIP entry point versioned hip_7.1 or
    later (hipStreamGetId, say) makes the dlopen fail there.  Every undefined HIP symbol's version <= 7.0."""
    import re
    out = subprocess.run(["nm", "-D", "--with-symbol-versions", "--undefined-only", _lib.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    vers = set(re.findall(r"@+hip_(\d+)\.(\d+)", out))
    assert vers, "no versioned HIP symbols found"
    too_new = sorted(v for v in vers if (int(v[0]), int(v[1])) > (7, 0))
    assert not too_new, too_new


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


def test_receipt_preimage_matches_oracle_restatement(oracle):
    """TarsHashable.h:43-75 field order, host mirror vs the oracle's independent restatement."""
    logs = [bcos_gpu.LogEntry(address="0x" + "11" * 20, topic=[b"\x01" * 32, b"\x02" * 32], data=b"xyz"),
            bcos_gpu.LogEntry(address="", topic=[], data=b"")]
    r = bcos_gpu.TransactionReceiptData(version=0, gas_used="21000", contract_address="", status=-1,
                                        output=b"\x00\x01", log_entries=logs, block_number=77)
    want = oracle.receipt_preimage(0, "21000", "", -1, b"\x00\x01",
                                   [("0x" + "11" * 20, [b"\x01" * 32, b"\x02" * 32], b"xyz"), ("", [], b"")], 77)
    assert r.preimage() == want
    assert want[:4] == bytes(4) and want[4:9] == b"21000" and want[9:13] == b"\xff" * 4
    assert want[-8:] == (77).to_bytes(8, "big")


def test_oracle_ecrecover_vector(oracle, kat):
    """EVMPrecompiledTest.cpp:58-72 through the precompile's input layout (Precompiled.cpp:443-482)."""
    h = bytes.fromhex("38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e")
    s = bytes.fromhex("789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02")
    inp = h + (27).to_bytes(32, "big") + h + s
    assert oracle.ecrecover(inp).hex() == "00" * 12 + "ceaccac640adf55b2028469bd36ba501f28b699d"
    assert oracle.ecrecover(h + (29).to_bytes(32, "big") + h + s) == b""
    # only the last byte of v is read: (1 << 8) + 27 behaves as 27
    assert oracle.ecrecover(h + ((1 << 8) + 27).to_bytes(32, "big") + h + s) == oracle.ecrecover(inp)


def test_native_preimage_packer(oracle):
    """bcosgpu_pack_tx_preimages (host C++) == the Python mirror == the oracle's restatement of
    TarsHashable.h:29-40, for ragged batches incl. empty fields, negative version / blockLimit and a
    batch large enough to take the threaded path."""
    from bcos_gpu import tx
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 20000):
        datas = []
        for i in range(n):
            datas.append(bcos_gpu.TransactionData(
                version=int(rng.integers(-2, 3)), chain_id="chain%d" % (i % 3) if i % 5 else "",
                group_id="group0", block_limit=int(rng.integers(-10, 10**12)), nonce=str(int(rng.integers(0, 10**18))),
                to=rng.bytes(20).hex() if i % 4 else "", input=rng.bytes(int(rng.integers(0, 300))),
                abi="" if i % 7 else "[{}]"))
        data, off = tx.pack_preimages(datas)
        assert len(off) == n + 1 and int(off[-1]) == len(data)
        for i in (list(range(min(n, 50))) + ([n - 1] if n else [])):
            d = datas[i]
            got = data[int(off[i]):int(off[i + 1])].tobytes()
            assert got == d.preimage() == oracle.tx_preimage(d.version, d.chain_id, d.group_id, d.block_limit,
                                                             d.nonce, d.to, d.input, d.abi)
