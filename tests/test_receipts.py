"""calculateReceiptRoot (BlockImpl.h:156-183) through the C ABI: the host receipt packer
(bcosgpu_pack_receipt_preimages, TarsHashable.h:54-73), the dataHash short-circuit (:47-51) and the
many-block receipt roots (bcosgpu_receipt_roots) -- from Python (ctypes views) and from C++
(tests/cpp/receipt_test.cpp over include/bcos_gpu.hpp calculateReceiptRoots), against the oracle's
restatement (oracle.receipt_preimage + oracle hashes + oracle.merkle).  Parity unpinned: the reference
holds no receipt-hash fixture; the field order is pinned to TarsHashable.h:54-73 only."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "fisco-bcos_amd", "lib")


def make_receipts(seed, block_sizes, data_hash_frac=0.1):
    """Seeded receipts: 0-3 logs of 0-4 topics (32 B, plus odd lengths), outputs 0-200 B, some dataHash
    set (32 B, and one short one); returns (list of bcos_gpu.TransactionReceipt, block_off)."""
    import bcos_gpu
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(sum(block_sizes)):
        logs = []
        for _ in range(int(rng.integers(0, 4))):
            topics = [rng.bytes(32 if rng.random() < 0.9 else int(rng.integers(0, 40)))
                      for _ in range(int(rng.integers(0, 5)))]
            logs.append(bcos_gpu.LogEntry(address=("0x" + rng.bytes(20).hex()) if rng.random() < 0.8 else "",
                                          topic=topics, data=rng.bytes(int(rng.integers(0, 100)))))
        d = bcos_gpu.TransactionReceiptData(
            version=int(rng.integers(0, 3)), gas_used=str(int(rng.integers(0, 10 ** 9))),
            contract_address=("0x" + rng.bytes(20).hex()) if rng.random() < 0.2 else "",
            status=int(rng.integers(-2, 20)), output=rng.bytes(int(rng.integers(0, 200))), log_entries=logs,
            block_number=int(rng.integers(0, 2 ** 40)))
        dh = b""
        u = rng.random()
        if u < data_hash_frac:
            dh = rng.bytes(32)
        elif u < data_hash_frac * 1.1:
            dh = rng.bytes(int(rng.integers(1, 32)))
        out.append(bcos_gpu.TransactionReceipt(data=d, data_hash=dh))
    bo = np.concatenate([[0], np.cumsum(block_sizes)]).astype(np.uint64)
    return out, bo


def oracle_expect(oracle, receipts, bo):
    pre = []
    for r in receipts:
        d = r.data
        pre.append(b"" if r.data_hash else oracle.receipt_preimage(
            d.version, d.gas_used, d.contract_address, d.status, d.output,
            [(lg.address, lg.topic or [], lg.data) for lg in d.log_entries or []], d.block_number))
    out = {}
    for hasher in (oracle.KECCAK256, oracle.SM3):
        hs = [bytes(r.data_hash).ljust(32, b"\0") if r.data_hash else oracle.hash_(hasher, p)
              for r, p in zip(receipts, pre)]
        roots = []
        for b in range(len(bo) - 1):
            blk = hs[int(bo[b]):int(bo[b + 1])]
            roots.append(oracle.merkle(hasher, 2, np.frombuffer(b"".join(blk), np.uint8).reshape(-1, 32))
                         if blk else bytes(32))
        out[hasher] = (hs, roots)
    return pre, out


def write_fixture(path, receipts, bo, pre, exp, oracle):
    def bs(b):
        b = bytes(b)
        return struct.pack("<I", len(b)) + b
    w = [b"RCPT", struct.pack("<I", len(bo) - 1), np.asarray(bo, dtype="<u8").tobytes()]
    for r in receipts:
        d = r.data
        w += [struct.pack("<i", d.version), bs(d.gas_used.encode()), bs(d.contract_address.encode()),
              struct.pack("<i", d.status), bs(d.output), struct.pack("<I", len(d.log_entries or []))]
        for lg in d.log_entries or []:
            w += [bs(lg.address.encode()), struct.pack("<I", len(lg.topic or []))]
            w += [bs(t) for t in lg.topic or []]
            w.append(bs(lg.data))
        w += [struct.pack("<q", d.block_number), bs(r.data_hash)]
    w += [bs(p) for p in pre]
    for hasher in (oracle.KECCAK256, oracle.SM3):
        hs, roots = exp[hasher]
        w += [b"".join(hs), b"".join(roots)]
    with open(path, "wb") as f:
        f.write(b"".join(w))


def _build(tmp_path):
    exe = str(tmp_path / "receipt_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "receipt_test.cpp"), "-L" + LIBDIR, "-lbcosgpu",
                    "-Wl,-rpath," + LIBDIR], check=True)
    return exe


BLOCKS = [0, 1, 2, 3, 17, 0, 64, 1000, 5]


def _run_cpp(tmp_path, oracle):
    receipts, bo = make_receipts(11, BLOCKS)
    pre, exp = oracle_expect(oracle, receipts, bo)
    fx = str(tmp_path / "receipts.bin")
    write_fixture(fx, receipts, bo, pre, exp, oracle)
    return subprocess.run([_build(tmp_path), fx], capture_output=True, text=True, timeout=300)


def test_receipt_packer_cpp_matches_oracle(tmp_path, oracle):
    """The C packer through C++ views: every preimage byte-equal to the restatement (no GPU needed)."""
    r = _run_cpp(tmp_path, oracle)
    assert r.returncode in (0, 77), r.stdout + r.stderr


def test_receipt_packer_python_views(oracle):
    import bcos_gpu
    from bcos_gpu import tx
    receipts, bo = make_receipts(5, [300])
    data, off = tx.pack_receipt_preimages(receipts)
    for i, r in enumerate(receipts):
        d = r.data
        want = b"" if r.data_hash else oracle.receipt_preimage(
            d.version, d.gas_used, d.contract_address, d.status, d.output,
            [(lg.address, lg.topic or [], lg.data) for lg in d.log_entries or []], d.block_number)
        assert data[int(off[i]):int(off[i + 1])].tobytes() == want
    assert bcos_gpu is not None


@pytest.mark.gpu
def test_receipt_roots_cpp_on_gpu(tmp_path, oracle, gpu):
    r = _run_cpp(tmp_path, oracle)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "receipt_test: ok" in r.stdout


@pytest.mark.gpu
def test_receipt_roots_abi_vs_oracle(oracle, gpu):
    """bcosgpu_receipt_roots from Python for both hashers, with and without dataHash receipts, incl. empty
    blocks; the per-receipt hashes it returns, too."""
    from bcos_gpu import tx
    for frac in (0.0, 0.3):
        receipts, bo = make_receipts(23, BLOCKS + [4096], data_hash_frac=frac)
        _, exp = oracle_expect(oracle, receipts, bo)
        for hasher in (oracle.KECCAK256, oracle.SM3):
            roots, hashes = tx.receipt_roots(hasher, receipts, bo)
            want_h, want_r = exp[hasher]
            assert [bytes(h) for h in hashes] == want_h
            assert [bytes(r) for r in roots] == want_r
