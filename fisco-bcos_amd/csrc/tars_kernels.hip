// tars_kernels.hip -- device-side decode of Tars-encoded transactions, so the
// createTransaction hot path runs from raw network bytes to verdicts without a host round trip:
//   TransactionFactoryImpl::createTransaction(txData, checkSig)  bcos-tars-protocol/.../protocol/TransactionFactoryImpl.h:46-85
//     -> TransactionImpl::decode (TransactionImpl.cpp:38-41, TarsSerializable.h:28-35: readFrom on a
//        tars::TarsInputStream over the bytes) -> calculateHash -> verify
// The wire format is tarscpp's (vcpkg dependency tarscpp >= 3.0.3-m, vcpkg.json:36-39; absent from the
// reference tree), restated from its published TarsInputStream rules:
//   head      1 byte (tag << 4 | type), or 0xF0 | type followed by the tag byte when tag >= 15
//   ints      ZeroTag(12) = 0, Char(0) 1 B, Short(1) 2 B, Int32(2) 4 B, Int64(3) 8 B, big-endian, signed
//   strings   String1(6): u8 length, String4(7): be32 length, then the bytes
//   vector<byte> SimpleList(13): head(Char, tag 0), an int (tag 0) length, then the bytes
//   struct    StructBegin(10) ... StructEnd(11); fields in tag order, absent optional fields = default;
//             unknown fields are skipped by type (Float 4 B, Double 8 B, Map/List: int count + elements)
//   readFrom  tars2cpp code reads each field with skipToTag(tag): skip smaller tags, stop before a larger
//             tag or a StructEnd; running off the buffer there means "absent", elsewhere it is an error
// bcostars::Transaction (tars/Transaction.tars:13-22): 1 data (struct TransactionData), 2 dataHash,
// 3 signature, 4 importTime, 5 attribute, 7 sender, 8 extraData.  TransactionData (:2-11): 1 version,
// 2 chainID, 3 groupID, 4 blockLimit, 5 nonce, 6 to, 7 input, 8 abi.  createTransaction clears dataHash
// and recomputes the hash (TransactionFactoryImpl.h:52-60); it is compared only under checkHash (:62-78).
// Pipeline: decode (one tx per lane: field offsets + lengths) -> exclusive scans of preimage and
// signature lengths (hipCUB) -> pack (preimage be32(version)|chainID|groupID|be64(blockLimit)|nonce|to|
// input|abi and signature into the SoA layout of bcosgpu_tx_verify_batch_dev) -> tx verify.
#include <hipcub/hipcub.hpp>
#include "engine.h"
#include "tars_decode.h"

namespace bcosgpu {

using namespace tars;

__global__ __launch_bounds__(256) void tars_tx_decode_kernel(const uint8_t* __restrict__ enc,
                                                             const uint64_t* __restrict__ enc_off, uint64_t n,
                                                             TxFields* __restrict__ fields,
                                                             uint64_t* __restrict__ pre_len,
                                                             uint64_t* __restrict__ sig_len,
                                                             uint8_t* __restrict__ dec_status) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    TxFields f;
    const bool ok = decode_tx(enc, enc_off[i], enc_off[i + 1], f);
    if (!ok) {
        for (int k = 0; k < F_N; ++k) f.len[k] = 0;
        f.version = 0;
        f.block_limit = 0;
    }
    fields[i] = f;
    pre_len[i] = ok ? 12ull + f.len[F_CHAIN] + f.len[F_GROUP] + f.len[F_NONCE] + f.len[F_TO] + f.len[F_INPUT] +
                          f.len[F_ABI]
                    : 0ull;
    sig_len[i] = ok ? f.len[F_SIG] : 0ull;
    dec_status[i] = ok ? 0 : 2;
}

// Pack: a team of kPackTeam lanes per tx writes its preimage / signature bytes, consecutive lanes on
// consecutive bytes, so the loads from the encoding and the stores to the packed buffers coalesce (one
// lane per tx walking its own bytes touched a different cache line per lane per byte).
constexpr int kPackTeam = 16;

__global__ __launch_bounds__(256) void tars_tx_pack_kernel(const uint8_t* __restrict__ enc, uint64_t n,
                                                           const TxFields* __restrict__ fields,
                                                           const uint64_t* __restrict__ pre_off,
                                                           const uint64_t* __restrict__ sig_off,
                                                           const uint8_t* __restrict__ dec_status,
                                                           uint8_t* __restrict__ pre, uint8_t* __restrict__ sig) {
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t i = t / kPackTeam;
    const uint32_t l = static_cast<uint32_t>(t % kPackTeam);
    if (i >= n || dec_status[i]) return;
    const TxFields f = fields[i];
    // preimage segments: be32(version) | chainID | groupID | be64(blockLimit) | nonce | to | input | abi
    const uint32_t e0 = 4, e1 = e0 + f.len[F_CHAIN], e2 = e1 + f.len[F_GROUP], e3 = e2 + 8,
                   e4 = e3 + f.len[F_NONCE], e5 = e4 + f.len[F_TO], e6 = e5 + f.len[F_INPUT], e7 = e6 + f.len[F_ABI];
    const uint32_t v = static_cast<uint32_t>(f.version);
    const uint64_t bl = static_cast<uint64_t>(f.block_limit);
    uint8_t* o = pre + pre_off[i];
    for (uint32_t j = l; j < e7; j += kPackTeam) {
        uint8_t x;
        if (j < e0) {
            x = static_cast<uint8_t>(v >> (24 - 8 * j));
        } else if (j >= e2 && j < e3) {
            x = static_cast<uint8_t>(bl >> (56 - 8 * (j - e2)));
        } else {
            uint64_t src;
            if (j < e1) src = f.off[F_CHAIN] + (j - e0);
            else if (j < e2) src = f.off[F_GROUP] + (j - e1);
            else if (j < e4) src = f.off[F_NONCE] + (j - e3);
            else if (j < e5) src = f.off[F_TO] + (j - e4);
            else if (j < e6) src = f.off[F_INPUT] + (j - e5);
            else src = f.off[F_ABI] + (j - e6);
            x = enc[src];
        }
        o[j] = x;
    }
    uint8_t* so = sig + sig_off[i];
    const uint8_t* si = enc + f.off[F_SIG];
    for (uint32_t j = l; j < f.len[F_SIG]; j += kPackTeam) so[j] = si[j];
}

// createTransaction's verdict order (TransactionFactoryImpl.h:46-84): the decode throws (2), then with
// checkHash a non-empty dataHash that differs from the recomputed hash throws (3, :62-78), then verify (1).
// Eight lanes per tx compare four bytes each; a wave ballot combines them.
__global__ __launch_bounds__(256) void tars_finish_kernel(const uint8_t* __restrict__ enc,
                                                          const TxFields* __restrict__ fields,
                                                          const uint8_t* __restrict__ dec,
                                                          const uint8_t* __restrict__ txhash,
                                                          uint8_t* __restrict__ status, uint64_t n, int check_hash) {
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t i = t / 8;
    const uint32_t l = static_cast<uint32_t>(t % 8);
    bool differs = false;
    uint8_t d = 0;
    if (i < n) {
        d = dec[i];
        if (!d && check_hash) {
            const uint32_t len = fields[i].len[F_HASH];
            if (len == 32) {
                const uint8_t* h = enc + fields[i].off[F_HASH] + 4 * l;
                const uint32_t want = reinterpret_cast<const uint32_t*>(txhash + 32 * i)[l];
                const uint32_t got = h[0] | (h[1] << 8) | (h[2] << 16) | (static_cast<uint32_t>(h[3]) << 24);
                differs = got != want;
            } else if (len != 0) {
                differs = true;
            }
        }
    }
    const uint64_t bad = __ballot(differs);  // every lane of the wave reaches this
    const uint32_t lane = threadIdx.x & 63;
    if (i >= n || l != 0) return;
    if (d) status[i] = d;
    else if ((bad >> lane) & 0xffull) status[i] = 3;
}

// Work buffer: fields[n] | pre_len[n] | sig_len[n] | dec_status[n] | scan temp storage
static size_t scan_temp_bytes(uint64_t n) {
    size_t t = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, static_cast<const uint64_t*>(nullptr),
                                           static_cast<uint64_t*>(nullptr), static_cast<int>(n));
    return t;
}

uint64_t tars_decode_work_bytes(uint64_t n) {
    const uint64_t a = (n * sizeof(TxFields) + 255) & ~255ull;
    const uint64_t b = (n * 8 + 255) & ~255ull;
    return a + 3 * b + scan_temp_bytes(n ? n : 1) + 256;
}

int launch_tars_tx_decode(const uint8_t* d_enc, const uint64_t* d_enc_off, uint64_t n, uint8_t* d_pre,
                          uint64_t* d_pre_off, uint8_t* d_sig, uint64_t* d_sig_off, uint8_t* d_dec_status,
                          void* d_work, uint64_t work_bytes, hipStream_t st) {
    if (n == 0) return 0;
    if (n > 0x7fffffffull || work_bytes < tars_decode_work_bytes(n)) return BCOSGPU_E_ARG;
    uint8_t* w = static_cast<uint8_t*>(d_work);
    TxFields* fields = reinterpret_cast<TxFields*>(w);
    w += (n * sizeof(TxFields) + 255) & ~255ull;
    uint64_t* pre_len = reinterpret_cast<uint64_t*>(w);
    w += (n * 8 + 255) & ~255ull;
    uint64_t* sig_len = reinterpret_cast<uint64_t*>(w);
    w += (n * 8 + 255) & ~255ull;
    if (!d_dec_status) d_dec_status = w;  // the internal status slot (tars_finish reads it from there)
    w += (n * 8 + 255) & ~255ull;
    size_t temp = scan_temp_bytes(n);
    const unsigned grid = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(tars_tx_decode_kernel, dim3(grid), dim3(256), 0, st, d_enc, d_enc_off, n, fields, pre_len,
                       sig_len, d_dec_status);
    if (hipMemsetAsync(d_pre_off, 0, 8, st) != hipSuccess || hipMemsetAsync(d_sig_off, 0, 8, st) != hipSuccess)
        return BCOSGPU_E_HIP;
    if (hipcub::DeviceScan::InclusiveSum(w, temp, pre_len, d_pre_off + 1, static_cast<int>(n), st) != hipSuccess ||
        hipcub::DeviceScan::InclusiveSum(w, temp, sig_len, d_sig_off + 1, static_cast<int>(n), st) != hipSuccess)
        return BCOSGPU_E_HIP;
    hipLaunchKernelGGL(tars_tx_pack_kernel, dim3(static_cast<unsigned>((n * kPackTeam + 255) / 256)), dim3(256), 0, st,
                       d_enc, n, fields, d_pre_off, d_sig_off,
                       d_dec_status, d_pre, d_sig);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_tars_finish(const uint8_t* d_enc, const void* d_work, const uint8_t* d_dec, const uint8_t* d_txhash,
                       uint8_t* d_status, uint64_t n, int check_hash, hipStream_t st) {
    if (n == 0) return 0;
    const uint8_t* w = static_cast<const uint8_t*>(d_work);
    const TxFields* fields = reinterpret_cast<const TxFields*>(w);
    if (!d_dec) d_dec = w + ((n * sizeof(TxFields) + 255) & ~255ull) + 2 * ((n * 8 + 255) & ~255ull);
    hipLaunchKernelGGL(tars_finish_kernel, dim3(static_cast<unsigned>((n * 8 + 255) / 256)), dim3(256), 0, st, d_enc,
                       fields, d_dec, d_txhash, d_status, n, check_hash);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

}  // namespace bcosgpu
