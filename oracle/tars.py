"""CPU restatement of the Tars transaction decode -- TEST INFRASTRUCTURE ONLY (tests/ and smoke()).

Follows bcostars::Transaction::readFrom as tars2cpp generates it for
bcos-tars-protocol/bcos-tars-protocol/tars/Transaction.tars:2-22, on tarscpp's TarsInputStream (vcpkg
dependency `tarscpp` >= 3.0.3-m, vcpkg.json:36-39, absent from /root/reference -- restated from its
published rules):
  - each field is read with skipToTag(tag): heads with smaller tags are skipped by type, a larger tag or
    a StructEnd stops the search ("absent" -> the default value); running off the end of the buffer inside
    skipToTag is caught there (TarsDecodeEndException) and also means "absent";
  - every other error (type mismatch, bad length, running off the end while reading a found field)
    propagates: TransactionImpl::decode throws, createTransaction fails (status 2 here);
  - read(Int32) accepts ZeroTag / Char / Short / Int32, read(Int64) also Int64; read(string) String1 /
    String4 (<= 100 MiB); read(vector<char>) SimpleList only (head(Char, 0), Int32 length, bytes);
  - read(struct): StructBegin, readFrom, then skipToStructEnd.
Parity of this decoder is UNPINNED: the reference tree holds no Tars-encoded fixtures and tarscpp is not
available to run; the GPU decoder is checked against this restatement and the TarsWriter round trip.
"""
import struct

CHAR, SHORT, INT32, INT64, FLOAT, DOUBLE, STRING1, STRING4, MAP, LIST, STRUCT_BEGIN, STRUCT_END, ZERO_TAG, \
    SIMPLE_LIST = range(14)


class DecodeEnd(Exception):
    """tars::TarsDecodeEndException."""


class DecodeError(Exception):
    """Any other tars decode exception."""


class _In:
    def __init__(self, buf):
        self.b = bytes(buf)
        self.pos = 0

    def take(self, n):
        if n > len(self.b) - self.pos:
            raise DecodeEnd()
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return v

    def head(self):
        c = self.take(1)[0]
        tag, type_ = c >> 4, c & 15
        if tag == 15:
            tag = self.take(1)[0]
        return tag, type_

    def integer(self, type_, wide=True):
        if type_ == ZERO_TAG:
            return 0
        if type_ == CHAR:
            return struct.unpack(">b", self.take(1))[0]
        if type_ == SHORT:
            return struct.unpack(">h", self.take(2))[0]
        if type_ == INT32:
            return struct.unpack(">i", self.take(4))[0]
        if type_ == INT64 and wide:
            return struct.unpack(">q", self.take(8))[0]
        raise DecodeError("int type mismatch")

    def string(self, type_):
        if type_ == STRING1:
            n = self.take(1)[0]
        elif type_ == STRING4:
            n = struct.unpack(">I", self.take(4))[0]
            if n > 100 << 20:
                raise DecodeError("string too long")
        else:
            raise DecodeError("string type mismatch")
        return self.take(n)

    def simple_list(self, type_):
        if type_ != SIMPLE_LIST:
            raise DecodeError("vector<char> type mismatch")
        _, t = self.head()
        if t != CHAR:
            raise DecodeError("simple list element type")
        _, t = self.head()
        n = self.integer(t, wide=False)
        if n < 0:
            raise DecodeError("negative size")
        return self.take(n)

    def skip(self, type_, depth=0):
        """skipField(type); like the GPU decoder, more than 16 nested containers is an error."""
        if type_ in (LIST, MAP, STRUCT_BEGIN) and depth >= 16:
            raise DecodeError("nesting")
        if type_ == CHAR:
            self.take(1)
        elif type_ == SHORT:
            self.take(2)
        elif type_ in (INT32, FLOAT):
            self.take(4)
        elif type_ in (INT64, DOUBLE):
            self.take(8)
        elif type_ in (ZERO_TAG, STRUCT_END):
            pass
        elif type_ == STRING1:
            self.take(self.take(1)[0])
        elif type_ == STRING4:
            self.take(struct.unpack(">I", self.take(4))[0])
        elif type_ == SIMPLE_LIST:
            self.simple_list(type_)
        elif type_ in (LIST, MAP):
            _, t = self.head()
            n = self.integer(t, wide=False)
            if n < 0:
                raise DecodeError("negative size")
            for _ in range(n * (2 if type_ == MAP else 1)):
                _, t = self.head()
                self.skip(t, depth + 1)
        elif type_ == STRUCT_BEGIN:
            self.to_struct_end(depth + 1)
        else:
            raise DecodeError("unknown type")

    def to_struct_end(self, depth=0):
        while True:
            _, t = self.head()
            if t == STRUCT_END:
                return
            self.skip(t, depth)

    def seek(self, want):
        """skipToTag(want) -> the field's type, or None when absent."""
        try:
            while self.pos < len(self.b):
                save = self.pos
                tag, t = self.head()
                if t == STRUCT_END or tag >= want:
                    if tag == want:
                        return t
                    self.pos = save
                    return None
                self.skip(t)
        except DecodeEnd:
            self.pos = len(self.b)
        return None


def decode_transaction(buf):
    """bcostars::Transaction readFrom.  Returns a dict of the fields (bytes / ints) or raises
    DecodeError / DecodeEnd like the reference's decode."""
    r = _In(buf)
    tx = {"version": 0, "chain_id": b"", "group_id": b"", "block_limit": 0, "nonce": b"", "to": b"",
          "input": b"", "abi": b"", "data_hash": b"", "signature": b"", "import_time": 0, "attribute": 0,
          "sender": b"", "extra_data": b""}
    t = r.seek(1)
    if t is not None:
        if t != STRUCT_BEGIN:
            raise DecodeError("struct type mismatch")
        for tag, key, kind in ((1, "version", "i32"), (2, "chain_id", "s"), (3, "group_id", "s"),
                               (4, "block_limit", "i64"), (5, "nonce", "s"), (6, "to", "s"), (7, "input", "v"),
                               (8, "abi", "s")):
            t = r.seek(tag)
            if t is not None:
                tx[key] = _read(r, t, kind)
        r.to_struct_end()
    for tag, key, kind in ((2, "data_hash", "v"), (3, "signature", "v"), (4, "import_time", "i64"),
                           (5, "attribute", "i32"), (7, "sender", "v"), (8, "extra_data", "s")):
        t = r.seek(tag)
        if t is not None:
            tx[key] = _read(r, t, kind)
    return tx


def _read(r, t, kind):
    if kind == "i32":
        return r.integer(t, wide=False)
    if kind == "i64":
        return r.integer(t)
    if kind == "s":
        return r.string(t)
    return r.simple_list(t)


def preimage(tx):
    """impl_calculate's field order (TarsHashable.h:29-40) over a decoded transaction."""
    return (struct.pack(">i", tx["version"]) + tx["chain_id"] + tx["group_id"] + struct.pack(">q", tx["block_limit"])
            + tx["nonce"] + tx["to"] + tx["input"] + tx["abi"])


def create_transactions(suite, encoded, check_sig=True, check_hash=False):
    """createTransaction(txData, checkSig, checkHash) over a batch on the CPU (oracle.tx_verify_packed for
    hash + recover + sender; TransactionFactoryImpl.h:46-85).  Returns (txhash list, sender list, status
    list) with the GPU API's status codes; without check_sig the sender is zero and only the decode and
    the hash check set a status."""
    import numpy as np

    from . import oracle
    decoded, status = [], []
    for e in encoded:
        try:
            decoded.append(decode_transaction(e))
            status.append(0)
        except (DecodeError, DecodeEnd):
            decoded.append(None)
            status.append(2)
    pres = [preimage(d) if d else b"" for d in decoded]
    sigs = [d["signature"] if d else b"" for d in decoded]
    pre = np.frombuffer(b"".join(pres) or b"\0", dtype=np.uint8).copy()
    sig = np.frombuffer(b"".join(sigs) or b"\0", dtype=np.uint8).copy()
    pre_off = np.cumsum([0] + [len(p) for p in pres]).astype(np.uint64)
    sig_off = np.cumsum([0] + [len(s) for s in sigs]).astype(np.uint64)
    h, snd, st = oracle.tx_verify_packed(suite, pre, pre_off, sig, sig_off)
    out_status = []
    for i, d in enumerate(decoded):
        if d is None:
            out_status.append(2)
        elif check_hash and d["data_hash"] and d["data_hash"] != bytes(h[i]):
            out_status.append(3)
        else:
            out_status.append(int(st[i]) if check_sig else 0)
    if not check_sig:
        snd = np.zeros_like(snd)
    return [bytes(x) for x in h], [bytes(x) for x in snd], out_status
