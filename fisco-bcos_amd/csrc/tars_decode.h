// tars_decode.h -- the Tars transaction decoder shared by the decode kernel (tars_kernels.hip) and its
// host build (tools/tars_host.cpp, a test tool that lets the CPU suite fuzz this exact code against the
// restatement in oracle/tars.py).  Wire format and reference citations: tars_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TARS_HD __host__ __device__ __forceinline__

namespace bcosgpu {
namespace tars {

enum : uint32_t {
    kChar = 0, kShort = 1, kInt32 = 2, kInt64 = 3, kFloat = 4, kDouble = 5, kString1 = 6, kString4 = 7,
    kMap = 8, kList = 9, kStructBegin = 10, kStructEnd = 11, kZeroTag = 12, kSimpleList = 13
};
enum : int { F_CHAIN = 0, F_GROUP, F_NONCE, F_TO, F_INPUT, F_ABI, F_SIG, F_HASH, F_N };

struct TxFields {
    uint64_t off[F_N];
    uint32_t len[F_N];
    int32_t version;
    int64_t block_limit;
};

// Reader errors mirror tarscpp's two exception kinds: running off the end of the buffer
// (TarsDecodeEndException: eof = true) and everything else (type mismatch, bad length).  Both end the
// decode, except inside seek() (skipToTag), which catches the end-of-buffer kind and reports the field
// absent.
struct Reader {
    const uint8_t* p;
    uint64_t pos, end;
    bool ok, eof;
    TARS_HD void overrun() {
        ok = false;
        eof = true;
    }
    TARS_HD uint32_t u8() {
        if (pos >= end) {
            overrun();
            return 0;
        }
        return p[pos++];
    }
    TARS_HD uint64_t be(int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | u8();
        return v;
    }
    TARS_HD void head(uint32_t& tag, uint32_t& type) {
        const uint32_t b = u8();
        type = b & 15u;
        tag = b >> 4;
        if (tag == 15u) tag = u8();
    }
    // read(Int64&) accepts every integer type; read(Int32&) (wide = false) rejects Int64
    TARS_HD int64_t integer(uint32_t type, bool wide = true) {
        switch (type) {
            case kZeroTag: return 0;
            case kChar: return static_cast<int8_t>(u8());
            case kShort: return static_cast<int16_t>(be(2));
            case kInt32: return static_cast<int32_t>(be(4));
            case kInt64:
                if (wide) return static_cast<int64_t>(be(8));
                [[fallthrough]];
            default: ok = false; return 0;
        }
    }
    TARS_HD void bytes(uint64_t n) {
        if (n > end - pos) overrun();
        else pos += n;
    }
    // read(std::string&): String1 / String4 (length <= TARS_MAX_STRING_LENGTH, 100 MiB)
    TARS_HD void string(uint32_t type, uint64_t& off, uint32_t& len) {
        uint64_t n = 0;
        if (type == kString1) n = u8();
        else if (type == kString4) n = static_cast<uint32_t>(be(4));
        else ok = false;
        if (n > (100ull << 20)) ok = false;
        off = pos;
        len = static_cast<uint32_t>(n);
        if (ok) bytes(n);
    }
    // read(std::vector<char>&): SimpleList only -- head(Char, 0), an Int32 length (tag 0), the bytes
    TARS_HD void simple_list(uint32_t type, uint64_t& off, uint32_t& len) {
        if (type != kSimpleList) {
            ok = false;
            return;
        }
        uint32_t t2, ty2;
        head(t2, ty2);
        if (ok && ty2 != kChar) ok = false;
        uint32_t t3, ty3;
        if (ok) head(t3, ty3);
        const int64_t n = ok ? integer(ty3, false) : 0;
        if (n < 0) ok = false;
        off = pos;
        len = static_cast<uint32_t>(n);
        if (ok) bytes(static_cast<uint64_t>(n));
    }
    // skipField(type): one value; lists / maps / structs nest through an explicit stack
    TARS_HD void skip(uint32_t type) {
        uint64_t rem[16];  // list / map frames: elements left; struct frames: ~0.  Nesting deeper than 16
                           // containers is rejected (tarscpp recurses without a limit)
        int sp = 0;
        // terminates: every pass consumes a head byte or pops a frame pushed by one
        while (ok) {
            switch (type) {  // consume one value
                case kChar: bytes(1); break;
                case kShort: bytes(2); break;
                case kInt32: case kFloat: bytes(4); break;
                case kInt64: case kDouble: bytes(8); break;
                case kZeroTag: break;
                case kString1: bytes(u8()); break;
                case kString4: bytes(static_cast<uint32_t>(be(4))); break;
                case kSimpleList: {
                    uint64_t o;
                    uint32_t l;
                    simple_list(type, o, l);
                    break;
                }
                case kList: case kMap: {
                    if (sp == 16) {
                        ok = false;
                        break;
                    }
                    uint32_t t3, ty3;
                    head(t3, ty3);
                    const int64_t n = ok ? integer(ty3, false) : 0;
                    if (!ok) break;
                    if (n < 0) ok = false;  // elements are then read (and may run off the end) one by one
                    else rem[sp++] = static_cast<uint64_t>(n) * (type == kMap ? 2u : 1u);
                    break;
                }
                case kStructBegin:
                    if (sp == 16) ok = false;
                    else rem[sp++] = ~0ull;
                    break;
                case kStructEnd: break;  // skipField(StructEnd) is a no-op
                default: ok = false;     // types 14, 15
            }
            for (;;) {  // advance to the next value to consume
                if (!ok || sp == 0) return;
                uint32_t tag;
                if (rem[sp - 1] == ~0ull) {  // inside a struct: next member or its end
                    head(tag, type);
                    if (ok && type == kStructEnd) {
                        --sp;
                        continue;
                    }
                    break;
                }
                if (rem[sp - 1] == 0) {
                    --sp;
                    continue;
                }
                --rem[sp - 1];
                head(tag, type);
                break;
            }
        }
    }
    // skipToTag(want): skip fields with smaller tags; stop before a larger tag or a StructEnd.  Running
    // off the end here (including inside a skipped field) means the field is absent, and so is every
    // later one (the reader is then at or past the end).
    TARS_HD bool seek(uint32_t want, uint32_t& type) {
        while (ok) {  // each pass consumes at least the head byte
            if (pos >= end) return false;
            const uint64_t save = pos;
            uint32_t tag;
            head(tag, type);
            if (ok && (type == kStructEnd || tag >= want)) {
                if (tag == want) return true;
                pos = save;
                return false;
            }
            if (ok) skip(type);
            if (!ok && eof) {
                ok = true;
                eof = false;
                pos = end;
                return false;
            }
        }
        return false;
    }
    // skipToStructEnd: members up to and including the StructEnd
    TARS_HD void to_struct_end() {
        while (ok) {
            uint32_t tag, type;
            head(tag, type);
            if (!ok || type == kStructEnd) return;
            skip(type);
        }
    }
};

// bcostars::TransactionData::readFrom (tars2cpp: one _is.read(field, tag, false) per field in tag order)
// followed by the skipToStructEnd of read(struct)
TARS_HD void read_tx_data(Reader& r, TxFields& f) {
    uint32_t type;
    if (r.seek(1, type)) f.version = static_cast<int32_t>(r.integer(type, false));
    if (r.ok && r.seek(2, type)) r.string(type, f.off[F_CHAIN], f.len[F_CHAIN]);
    if (r.ok && r.seek(3, type)) r.string(type, f.off[F_GROUP], f.len[F_GROUP]);
    if (r.ok && r.seek(4, type)) f.block_limit = r.integer(type);
    if (r.ok && r.seek(5, type)) r.string(type, f.off[F_NONCE], f.len[F_NONCE]);
    if (r.ok && r.seek(6, type)) r.string(type, f.off[F_TO], f.len[F_TO]);
    if (r.ok && r.seek(7, type)) r.simple_list(type, f.off[F_INPUT], f.len[F_INPUT]);
    if (r.ok && r.seek(8, type)) r.string(type, f.off[F_ABI], f.len[F_ABI]);
    if (r.ok) r.to_struct_end();
}


// bcostars::Transaction::readFrom over enc[begin, end): field offsets / lengths into f; false when the
// reference's decode would throw
TARS_HD bool decode_tx(const uint8_t* enc, uint64_t begin, uint64_t end, TxFields& f) {
    Reader r{enc, begin, end, true, false};
    for (int k = 0; k < F_N; ++k) {
        f.off[k] = 0;
        f.len[k] = 0;
    }
    f.version = 0;
    f.block_limit = 0;
    // bcostars::Transaction::readFrom: every field is optional and read (type-checked) in tag order;
    // only data (1) and signature (3) feed the verify, dataHash (2) is discarded by createTransaction
    uint32_t type;
    uint64_t o;
    uint32_t l;
    if (r.seek(1, type)) {
        if (type != kStructBegin) r.ok = false;
        else read_tx_data(r, f);
    }
    if (r.ok && r.seek(2, type)) r.simple_list(type, f.off[F_HASH], f.len[F_HASH]);  // dataHash
    if (r.ok && r.seek(3, type)) r.simple_list(type, f.off[F_SIG], f.len[F_SIG]);
    if (r.ok && r.seek(4, type)) (void)r.integer(type);                        // importTime (long)
    if (r.ok && r.seek(5, type)) (void)r.integer(type, false);                 // attribute (int)
    if (r.ok && r.seek(7, type)) r.simple_list(type, o, l);                   // sender
    if (r.ok && r.seek(8, type)) r.string(type, o, l);                         // extraData
    return r.ok;
}

}  // namespace tars
}  // namespace bcosgpu
