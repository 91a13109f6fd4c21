"""Tars-encoded transactions: the encoder side (host) and the batched createTransaction (GPU).

  bcostars::Transaction / TransactionData    bcos-tars-protocol/bcos-tars-protocol/tars/Transaction.tars:2-22
  TransactionImpl::encode / decode           bcos-tars-protocol/bcos-tars-protocol/protocol/TransactionImpl.cpp:38-46
      (impl/TarsSerializable.h:16-35: tars::TarsOutputStream / TarsInputStream over the struct)
  TransactionFactoryImpl::createTransaction  bcos-tars-protocol/bcos-tars-protocol/protocol/TransactionFactoryImpl.h:46-85
      decode -> clear dataHash, recompute the hash (:52-60) -> checkHash (:62-78) -> verify (:80-83)

The wire format belongs to tarscpp (vcpkg dependency `tarscpp` >= 3.0.3-m, vcpkg.json:36-39), which is
not in the reference tree; TarsWriter restates its TarsOutputStream rules (minimal integer encoding,
String1 / String4, SimpleList for vector<byte>, StructBegin / StructEnd) and tars2cpp's writeTo (optional
fields equal to their default are not written).  The decode runs on the GPU
(fisco-bcos_amd/csrc/tars_kernels.hip); tests check it against the CPU restatement in oracle/tars.py.
"""
import struct

import numpy as np

from ._lib import check, ensure_device, lib
from .crypto import CryptoSuite, _ptr, pack_messages
from .tx import Transaction, TransactionData

# tars::DataHead types (TarsType.h)
CHAR, SHORT, INT32, INT64, FLOAT, DOUBLE, STRING1, STRING4, MAP, LIST, STRUCT_BEGIN, STRUCT_END, ZERO_TAG, \
    SIMPLE_LIST = range(14)

STATUS_OK, STATUS_INVALID_SIGNATURE, STATUS_MALFORMED, STATUS_HASH_MISMATCH = 0, 1, 2, 3


class TarsWriter:
    """tars::TarsOutputStream<BufferWriter> (the subset the transaction structs use, plus the types an
    unknown field may carry)."""

    def __init__(self):
        self.buf = bytearray()

    def head(self, type_, tag):
        if tag < 15:
            self.buf.append((tag << 4) | type_)
        else:
            self.buf += bytes([0xF0 | type_, tag])

    def int(self, v, tag):
        """write(Char/Short/Int32/Int64): the narrowest type that holds v; 0 -> ZeroTag."""
        if v == 0:
            self.head(ZERO_TAG, tag)
        elif -128 <= v <= 127:
            self.head(CHAR, tag)
            self.buf += struct.pack(">b", v)
        elif -32768 <= v <= 32767:
            self.head(SHORT, tag)
            self.buf += struct.pack(">h", v)
        elif -2**31 <= v < 2**31:
            self.head(INT32, tag)
            self.buf += struct.pack(">i", v)
        else:
            self.head(INT64, tag)
            self.buf += struct.pack(">q", v)

    def string(self, s, tag):
        b = s.encode() if isinstance(s, str) else bytes(s)
        if len(b) > 255:
            self.head(STRING4, tag)
            self.buf += struct.pack(">I", len(b))
        else:
            self.head(STRING1, tag)
            self.buf.append(len(b))
        self.buf += b

    def bytes_(self, b, tag):
        """write(vector<char>): SimpleList, head(Char, 0), the Int32 length (tag 0), the bytes."""
        b = bytes(b)
        self.head(SIMPLE_LIST, tag)
        self.head(CHAR, 0)
        self.int(len(b), 0)
        self.buf += b

    def double(self, v, tag):
        self.head(DOUBLE, tag)
        self.buf += struct.pack(">d", v)

    def int_list(self, vs, tag):
        """write(vector<Int64>) as a List (an unknown field type the decoder must skip)."""
        self.head(LIST, tag)
        self.int(len(vs), 0)
        for v in vs:
            self.int(v, 0)

    def struct_begin(self, tag):
        self.head(STRUCT_BEGIN, tag)

    def struct_end(self):
        self.head(STRUCT_END, 0)


def write_tx_data(w: TarsWriter, d: TransactionData):
    """bcostars::TransactionData::writeTo (tars2cpp; Transaction.tars:2-11)."""
    if d.version != 0:
        w.int(d.version, 1)
    if d.chain_id:
        w.string(d.chain_id, 2)
    if d.group_id:
        w.string(d.group_id, 3)
    if d.block_limit != 0:
        w.int(d.block_limit, 4)
    if d.nonce:
        w.string(d.nonce, 5)
    if d.to:
        w.string(d.to, 6)
    if len(d.input):
        w.bytes_(d.input, 7)
    if d.abi:
        w.string(d.abi, 8)


def encode_transaction(tx: Transaction, data_hash=b"", import_time=0, attribute=0, extra_data="") -> bytes:
    """TransactionImpl::encode (TransactionImpl.cpp:43-46): bcostars::Transaction::writeTo
    (Transaction.tars:13-22; tag 6 `source` is commented out in the schema)."""
    w = TarsWriter()
    w.struct_begin(1)
    write_tx_data(w, tx.data)
    w.struct_end()
    if data_hash:
        w.bytes_(data_hash, 2)
    if tx.signature:
        w.bytes_(tx.signature, 3)
    if import_time:
        w.int(import_time, 4)
    if attribute:
        w.int(attribute, 5)
    if tx.sender:
        w.bytes_(tx.sender, 7)
    if extra_data:
        w.string(extra_data, 8)
    return bytes(w.buf)


def create_transactions(suite: CryptoSuite, encoded, check_sig=True, check_hash=False):
    """TransactionFactoryImpl::createTransaction(txData, checkSig, checkHash) over a batch, decode
    included, on the GPU (bcosgpu_tars_tx_verify_batch); sender is zero when not check_sig.  `encoded` is a list of bytes (or (data,
    offsets[n+1])).  Returns (txhash uint8[n,32], sender uint8[n,20], status uint8[n]); status 0 ok,
    1 InvalidSignature (verify throws, :80-83), 2 the Tars decode throws, 3 the dataHash mismatch check
    throws (:62-78)."""
    if isinstance(encoded, tuple):
        data, off = encoded
    else:
        data, off = pack_messages([bytes(e) for e in encoded])
    n = len(off) - 1
    txhash = np.zeros((n, 32), dtype=np.uint8)
    sender = np.zeros((n, 20), dtype=np.uint8)
    status = np.zeros(n, dtype=np.uint8)
    if n:
        ensure_device()
        d = data if len(data) else np.zeros(1, dtype=np.uint8)
        check(lib().bcosgpu_tars_tx_verify_batch(suite.suite, _ptr(d), _ptr(off), n, int(bool(check_sig)),
                                                 int(bool(check_hash)),
                                                 _ptr(txhash), _ptr(sender), _ptr(status)))
    return txhash, sender, status
