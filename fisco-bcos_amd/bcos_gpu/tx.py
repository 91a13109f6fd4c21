"""Transaction-side mirror: the tx-hash preimage and batched Transaction::verify.

  bcostars::TransactionData fields         bcos-tars-protocol/bcos-tars-protocol/tars/Transaction.tars:2-11
  impl_calculate<Hasher>(Transaction)      bcos-tars-protocol/bcos-tars-protocol/impl/TarsHashable.h:16-41
      H(be32(version) || chainID || groupID || be64(blockLimit) || nonce || to || input || abi)
  Transaction::verify                      bcos-framework/bcos-framework/protocol/Transaction.h:68-82
  TransactionSync::importDownloadedTxs     bcos-txpool/bcos-txpool/sync/TransactionSync.cpp:496-575
  BlockImpl::calculateTransactionRoot      bcos-tars-protocol/bcos-tars-protocol/protocol/BlockImpl.h:111-154
  bcostars::TransactionReceiptData         bcos-tars-protocol/bcos-tars-protocol/tars/TransactionReceipt.tars:2-23
  impl_calculate<Hasher>(TransactionReceipt) TarsHashable.h:43-75
      H(be32(version) || gasUsed || contractAddress || be32(status) || output
        || for each log: (address || topic_0 || ... || data) || be64(blockNumber))
  BlockImpl::calculateReceiptRoot          BlockImpl.h:156-183
"""
import ctypes
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, ensure_device, lib
from .crypto import CryptoSuite, Merkle, _ptr, pack_messages

STATUS_NONE = 0  # TransactionStatus::None
STATUS_INVALID_SIGNATURE = 1  # TransactionStatus::InvalidSignature (TxValidator.cpp:54-61)


@dataclass
class TransactionData:
    """bcostars::TransactionData (Transaction.tars:2-11)."""
    version: int = 0
    chain_id: str = ""
    group_id: str = ""
    block_limit: int = 0
    nonce: str = ""
    to: str = ""
    input: bytes = b""
    abi: str = ""

    def preimage(self) -> bytes:
        """The bytes impl_calculate feeds the hasher, in order (TarsHashable.h:29-40)."""
        return (struct.pack(">i", self.version) + self.chain_id.encode() + self.group_id.encode()
                + struct.pack(">q", self.block_limit) + self.nonce.encode() + self.to.encode()
                + bytes(self.input) + self.abi.encode())


@dataclass
class LogEntry:
    """bcostars::LogEntry (TransactionReceipt.tars:2-6)."""
    address: str = ""
    topic: list = None
    data: bytes = b""


@dataclass
class TransactionReceiptData:
    """bcostars::TransactionReceiptData (TransactionReceipt.tars:8-16)."""
    version: int = 0
    gas_used: str = ""
    contract_address: str = ""
    status: int = 0
    output: bytes = b""
    log_entries: list = None
    block_number: int = 0

    def preimage(self) -> bytes:
        """The bytes impl_calculate<Hasher>(TransactionReceipt) feeds the hasher (TarsHashable.h:54-73)."""
        parts = [struct.pack(">i", self.version), self.gas_used.encode(), self.contract_address.encode(),
                 struct.pack(">i", self.status), bytes(self.output)]
        for log in self.log_entries or []:
            parts.append(log.address.encode())
            parts.extend(bytes(t) for t in (log.topic or []))
            parts.append(bytes(log.data))
        parts.append(struct.pack(">q", self.block_number))
        return b"".join(parts)


@dataclass
class TransactionReceipt:
    """bcostars::TransactionReceipt (TransactionReceipt.tars:18-22); a non-empty data_hash
    short-circuits the hash (TarsHashable.h:47-51)."""
    data: TransactionReceiptData
    data_hash: bytes = b""


@dataclass
class Transaction:
    data: TransactionData
    signature: bytes = b""
    sender: bytes = b""

    def hash(self, suite: CryptoSuite) -> bytes:
        return suite.hash(self.data.preimage())


class _TxDataView(ctypes.Structure):
    """bcosgpu_TransactionData (include/bcos_gpu.h): pointers into the caller's fields."""
    _fields_ = [("version", ctypes.c_int32),
                ("chain_id", ctypes.c_char_p), ("chain_id_len", ctypes.c_size_t),
                ("group_id", ctypes.c_char_p), ("group_id_len", ctypes.c_size_t),
                ("block_limit", ctypes.c_int64),
                ("nonce", ctypes.c_char_p), ("nonce_len", ctypes.c_size_t),
                ("to", ctypes.c_char_p), ("to_len", ctypes.c_size_t),
                ("input", ctypes.c_char_p), ("input_len", ctypes.c_size_t),
                ("abi", ctypes.c_char_p), ("abi_len", ctypes.c_size_t)]


def pack_preimages(datas):
    """The native packer (bcosgpu_pack_tx_preimages, host C++): list[TransactionData] ->
    (uint8 packed preimages, uint64 offsets[n+1]) in the SoA layout bcosgpu_tx_verify_batch takes."""
    n = len(datas)
    views = (_TxDataView * max(n, 1))()
    keep = []
    for i, d in enumerate(datas):
        fields = [d.chain_id.encode(), d.group_id.encode(), d.nonce.encode(), d.to.encode(), bytes(d.input),
                  d.abi.encode()]
        keep.append(fields)
        v = views[i]
        v.version = d.version
        v.block_limit = d.block_limit
        for name, b in zip(("chain_id", "group_id", "nonce", "to", "input", "abi"), fields):
            setattr(v, name, b)
            setattr(v, name + "_len", len(b))
    size = int(lib().bcosgpu_tx_preimage_size(views, n))
    out = np.zeros(max(size, 1), dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    check(lib().bcosgpu_pack_tx_preimages(views, n, _ptr(out), size, _ptr(off)))
    return out[:size], off


def _outputs(n, out):
    """(txhash uint8[n,32], sender uint8[n,20], status uint8[n]): `out` (a caller's reused buffers, as a node
    keeps its batch arrays; at least n rows each) or fresh zeroed arrays."""
    if out is None:
        return np.zeros((n, 32), dtype=np.uint8), np.zeros((n, 20), dtype=np.uint8), np.zeros(n, dtype=np.uint8)
    txhash, sender, status = out
    assert txhash.shape[0] >= n and sender.shape[0] >= n and status.shape[0] >= n
    assert all(a.flags.c_contiguous and a.dtype == np.uint8 for a in out)
    return txhash[:n], sender[:n], status[:n]


def verify_packed(suite: CryptoSuite, pre, pre_off, sig, sig_off, out=None):
    """Batched Transaction::verify over packed buffers.
    Returns (txhash uint8[n,32], sender uint8[n,20], status uint8[n]) -- written into `out` when given."""
    n = len(pre_off) - 1
    txhash, sender, status = _outputs(n, out)
    if n:
        ensure_device()
        p = pre if len(pre) else np.zeros(1, dtype=np.uint8)
        s = sig if len(sig) else np.zeros(1, dtype=np.uint8)
        check(lib().bcosgpu_tx_verify_batch(suite.suite, _ptr(p), _ptr(pre_off), _ptr(s), _ptr(sig_off), n,
                                            _ptr(txhash), _ptr(sender), _ptr(status)))
    return txhash, sender, status


def _devices(devices):
    d = np.ascontiguousarray(devices, dtype=np.int32)
    assert d.ndim == 1 and 1 <= d.size <= 64, "device list: 1 to 64 entries"
    return d


def verify_packed_multi(devices, suite: CryptoSuite, pre, pre_off, sig, sig_off, width=None, out=None):
    """verify_packed over a device set in ONE process (bcosgpu_tx_verify_batch_multi): the batch split by
    index over `devices` (an index may repeat: two shards on one GPU, distinct streams).  With `width`,
    also the block's tx root (bcosgpu_block_verify_multi: per-GPU frontiers gathered on devices[0]).
    Returns (txhash, sender, status) or (txhash, sender, status, root)."""
    d = _devices(devices)
    n = len(pre_off) - 1
    txhash, sender, status = _outputs(n, out)
    p = pre if len(pre) else np.zeros(1, dtype=np.uint8)
    s = sig if len(sig) else np.zeros(1, dtype=np.uint8)
    po = np.ascontiguousarray(pre_off, dtype=np.uint64)
    so = np.ascontiguousarray(sig_off, dtype=np.uint64)
    if width is None:
        check(lib().bcosgpu_tx_verify_batch_multi(_ptr(d), d.size, suite.suite, _ptr(p), _ptr(po), _ptr(s), _ptr(so), n,
                                                  _ptr(txhash), _ptr(sender), _ptr(status)))
        return txhash, sender, status
    root = np.zeros(32, dtype=np.uint8)
    check(lib().bcosgpu_block_verify_multi(_ptr(d), d.size, suite.suite, _ptr(p), _ptr(po), _ptr(s), _ptr(so), n,
                                           width, _ptr(txhash), _ptr(sender), _ptr(status), _ptr(root)))
    return txhash, sender, status, root.tobytes()


def blocks_verify_multi(devices, suite: CryptoSuite, pre, pre_off, sig, sig_off, block_off, width=2, out=None):
    """Many blocks in one call over a device set (bcosgpu_blocks_verify_multi): block b = txs
    [block_off[b], block_off[b+1]).  Returns (txhash, sender, status, roots uint8[nblocks, 32])."""
    d = _devices(devices)
    bo = np.ascontiguousarray(block_off, dtype=np.uint64)
    nb = bo.size - 1
    n = int(bo[-1]) if nb >= 0 else 0
    txhash, sender, status = _outputs(max(n, 1), out)
    roots = np.zeros((max(nb, 1), 32), dtype=np.uint8)
    p = pre if len(pre) else np.zeros(1, dtype=np.uint8)
    s = sig if len(sig) else np.zeros(1, dtype=np.uint8)
    po = np.ascontiguousarray(pre_off, dtype=np.uint64)
    so = np.ascontiguousarray(sig_off, dtype=np.uint64)
    check(lib().bcosgpu_blocks_verify_multi(_ptr(d), d.size, suite.suite, _ptr(p), _ptr(po), _ptr(s), _ptr(so), _ptr(bo),
                                            nb, width, _ptr(txhash), _ptr(sender), _ptr(status), _ptr(roots)))
    return txhash[:n], sender[:n], status[:n], roots[:nb]


def merkle_root_multi(devices, hasher, width, leaves):
    """Merkle<H, width> root over a device set (bcosgpu_merkle_root_multi); leaves uint8[n, 32]."""
    d = _devices(devices)
    lv = np.ascontiguousarray(leaves, dtype=np.uint8).reshape(-1, 32)
    root = np.zeros(32, dtype=np.uint8)
    check(lib().bcosgpu_merkle_root_multi(_ptr(d), d.size, hasher, width, _ptr(lv if lv.size else np.zeros(32, np.uint8)),
                                          lv.shape[0], _ptr(root)))
    return root.tobytes()


def verify_transactions(suite: CryptoSuite, txs):
    """importDownloadedTxs' parallel loop (TransactionSync.cpp:516-548) on the GPU: every tx whose
    sender is unset is verified; tx.sender is set on success (Transaction.h:70-81).  Returns the
    per-tx status list."""
    todo = [i for i, t in enumerate(txs) if not t.sender]
    status = [STATUS_NONE] * len(txs)
    if not todo:
        return status
    pre, pre_off = pack_preimages([txs[i].data for i in todo])
    sig, sig_off = pack_messages([bytes(txs[i].signature) for i in todo])
    _, sender, st = verify_packed(suite, pre, pre_off, sig, sig_off)
    for k, i in enumerate(todo):
        if st[k] == 0:
            txs[i].sender = sender[k].tobytes()
        status[i] = int(st[k])
    return status


class _BytesView(ctypes.Structure):
    _fields_ = [("data", ctypes.c_char_p), ("len", ctypes.c_size_t)]


class _LogView(ctypes.Structure):
    """bcosgpu_LogEntry (include/bcos_gpu.h)."""
    _fields_ = [("address", ctypes.c_char_p), ("address_len", ctypes.c_size_t),
                ("topics", ctypes.POINTER(_BytesView)), ("ntopics", ctypes.c_size_t),
                ("data", ctypes.c_char_p), ("data_len", ctypes.c_size_t)]


class _ReceiptView(ctypes.Structure):
    """bcosgpu_TransactionReceiptData (include/bcos_gpu.h): pointers into the caller's fields."""
    _fields_ = [("version", ctypes.c_int32),
                ("gas_used", ctypes.c_char_p), ("gas_used_len", ctypes.c_size_t),
                ("contract_address", ctypes.c_char_p), ("contract_address_len", ctypes.c_size_t),
                ("status", ctypes.c_int32),
                ("output", ctypes.c_char_p), ("output_len", ctypes.c_size_t),
                ("logs", ctypes.POINTER(_LogView)), ("nlogs", ctypes.c_size_t),
                ("block_number", ctypes.c_int64),
                ("data_hash", ctypes.c_char_p), ("data_hash_len", ctypes.c_size_t)]


def _receipt_views(receipts):
    """ctypes views of TransactionReceipt objects; returns (views array, keep-alive list)."""
    n = len(receipts)
    views = (_ReceiptView * max(n, 1))()
    keep = []
    for i, r in enumerate(receipts):
        d, v = r.data, views[i]
        fields = [d.gas_used.encode(), d.contract_address.encode(), bytes(d.output), bytes(r.data_hash or b"")]
        keep.append(fields)
        v.version, v.status, v.block_number = d.version, d.status, d.block_number
        for name, b in zip(("gas_used", "contract_address", "output", "data_hash"), fields):
            setattr(v, name, b)
            setattr(v, name + "_len", len(b))
        logs = d.log_entries or []
        if logs:
            la = (_LogView * len(logs))()
            for k, lg in enumerate(logs):
                addr, data, topics = lg.address.encode(), bytes(lg.data), [bytes(t) for t in lg.topic or []]
                ta = (_BytesView * max(len(topics), 1))()
                for j, t in enumerate(topics):
                    ta[j].data, ta[j].len = t, len(t)
                keep.append((addr, data, topics, ta))
                la[k].address, la[k].address_len = addr, len(addr)
                la[k].data, la[k].data_len = data, len(data)
                la[k].topics, la[k].ntopics = ta, len(topics)
            keep.append(la)
            v.logs, v.nlogs = la, len(logs)
    return views, keep


def pack_receipt_preimages(receipts):
    """The native receipt packer (bcosgpu_pack_receipt_preimages, host C++): list[TransactionReceipt] ->
    (uint8 packed preimages, uint64 offsets[n+1]); a receipt with a dataHash gets an empty preimage."""
    views, keep = _receipt_views(receipts)
    n = len(receipts)
    size = int(lib().bcosgpu_receipt_preimage_size(views, n))
    out = np.zeros(max(size, 1), dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    check(lib().bcosgpu_pack_receipt_preimages(views, n, _ptr(out), size, _ptr(off)))
    del keep
    return out[:size], off


def receipt_roots(hasher, receipts, block_off):
    """bcosgpu_receipt_roots: calculateReceiptRoot for many blocks in one engine call (block b = receipts
    [block_off[b], block_off[b+1])).  Returns (roots uint8[nblocks, 32], receipt hashes uint8[n, 32])."""
    ensure_device()
    bo = np.ascontiguousarray(block_off, dtype=np.uint64)
    nb = bo.size - 1
    views, keep = _receipt_views(receipts)
    n = len(receipts)
    roots = np.zeros((max(nb, 1), 32), dtype=np.uint8)
    hashes = np.zeros((max(n, 1), 32), dtype=np.uint8)
    check(lib().bcosgpu_receipt_roots(hasher, views, _ptr(bo), nb, _ptr(roots), _ptr(hashes)))
    del keep
    return roots[:nb], hashes[:n]


def calculate_receipt_root(suite: CryptoSuite, receipts) -> bytes:
    """BlockImpl::calculateReceiptRoot (BlockImpl.h:156-183) through bcosgpu_receipt_roots: receipts packed
    by the native packer, hashed on the GPU (a set dataHash used as is, TarsHashable.h:47-51), width-2 root;
    no receipts -> the zero hash (:159-163)."""
    if len(receipts) == 0:
        return bytes(32)
    roots, _ = receipt_roots(suite.hash_impl.kind, receipts, [0, len(receipts)])
    return roots[0].tobytes()


def calculate_roots_batch(suite: CryptoSuite, blocks_of_hashes):
    """calculateTransactionRoot / calculateReceiptRoot for many blocks at once (one engine call,
    bcosgpu_merkle_roots_batch); each block is a list of 32-byte hashes, empty -> zero hash."""
    return Merkle(suite.hash_impl, 2).roots_batch(blocks_of_hashes)


def calculate_transaction_root(suite: CryptoSuite, tx_hashes) -> bytes:
    """BlockImpl::calculateTransactionRoot (BlockImpl.h:111-154): width-2 Merkle over the tx hashes;
    no transactions -> the zero hash (:116-119)."""
    if len(tx_hashes) == 0:
        return bytes(32)
    return Merkle(suite.hash_impl, 2).root(tx_hashes)
