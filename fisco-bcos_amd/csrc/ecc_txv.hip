// ecc_txv.hip -- the one-lane verification kernel tx_verify_kernel<suite, occupancy, field, IO> and
// launch_verify<IO>, which picks the kernel for a batch: the lane-trio / pair kernels (ecc_coop.hip,
// ecc_pair.hip) or the one-lane kernel at occupancy 1 or 2, by rounds x measured latency.  IO = TxIO is
// Transaction::verify (bcosgpu_tx_verify_batch*), IO = SigIO the reference-interface recover / SM2
// verify batches (bcosgpu_secp256k1_recover_batch*, bcosgpu_sm2_verify_batch*).
#include "ecc_device.h"

namespace bcosgpu {

// One tx (or signature) per lane: digest, recover / verify, address.
// OCC = waves per SIMD the register allocation must allow: 1 (no spills, lowest per-tx latency:
// small batches) or 2 (spills ~120 VGPRs to scratch but doubles the resident waves: large batches).
template <int SUITE, int OCC, bool F26, class IO>
__global__ __launch_bounds__(256, OCC) void tx_verify_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                             int tbits) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe h;
    io.template digest<SUITE == BCOSGPU_SUITE_SM2 ? SM3 : KECCAK256>(i, h);
    fe x, y, r, s;
    uint32_t ad[5] = {0, 0, 0, 0, 0};
    bool ok;
    // OCC 2: the variable-base table's x-coordinates live in LDS (16 KiB per wave, 128 KiB per CU
    // at 2 workgroups per CU), the rest of the working set in 256 VGPRs
    constexpr bool kLds = OCC == 2;
    __shared__ uint32_t ldsx_all[kLds ? 4 * 4096 : 1];
    uint32_t* ldsx = kLds ? ldsx_all + (threadIdx.x >> 6) * 4096 + (threadIdx.x & 63) : nullptr;
    if constexpr (SUITE == BCOSGPU_SUITE_SM2 && std::is_same_v<IO, KeyIO>) {
        uint32_t X[8], Y[8];
        io.sm2_sig(i, r, s, X, Y);  // r || s from the signature, the key from pub64
        if constexpr (F26) ok = sm2_verify_rs26<kLds>(h, r, s, X, Y, CombTab{tab, tbits}, x, y, ldsx);
        else ok = sm2_verify_rs<kLds>(h, r, s, X, Y, CombTab{tab, tbits}, x, y, ldsx);
        io.finish(i, ok, ad, nullptr, nullptr);
    } else if constexpr (SUITE == BCOSGPU_SUITE_SM2) {
        // (the r || s || pub parse inside the lane functions: the throughput kernels' register
        // allocation -- C3's spills -- depends on this form)
        const uint8_t* sp;
        const uint32_t slen = io.sig_span(i, sp);
        if constexpr (F26) ok = sm2_verify_lane26<kLds>(h, sp, slen, CombTab{tab, tbits}, x, y, ldsx);
        else ok = sm2_verify_lane<kLds>(h, sp, slen, CombTab{tab, tbits}, x, y, ldsx);
        if (ok && io.want_addr()) sm3_address(ad, x, y);
        io.finish(i, ok, ad, nullptr, nullptr);
    } else {
        uint32_t v;
        io.rsv(i, r, s, v);  // r = s = 0 for a malformed signature: the recovery rejects it
        if constexpr (F26) ok = secp256k1_recover_rsv26<kLds>(h, r, s, v, CombTab{tab, tbits}, x, y, ldsx);
        else ok = secp256k1_recover_rsv<kLds>(h, r, s, v, CombTab{tab, tbits}, x, y, ldsx);
        if (ok && io.want_addr()) keccak_address(ad, x, y);
        io.finish(i, ok, ad, &x, &y);
    }
}

// Every kernel runs its batch in rounds of resident workgroups -- the trio kernels take 40 txs per CU,
// the pair kernels 64, the one-lane kernel 256 at occupancy 1 (one wave per SIMD) and 512 at
// occupancy 2 -- and a round costs a fixed latency, so a kernel's cost is rounds x latency.  The
// occupancy-2 kernel's last round, when it leaves every SIMD at most one wave, has its own (shorter)
// latency.  Latencies relative to the trio kernel's round, fitted from the round-4 sweep on MI355X
// (tools/small_sweep.py -> tools/fit_auto.py, profiles/r04_small_sweep.json and _fit.json): secp256k1
// trio 0.379 / pair 0.485 / one-lane 1.00 (occupancy 1) / 1.70 (occupancy 2) / 0.97 ms (its single-wave
// round); SM2 0.593 / 0.996 / 1.42 / 2.56 / 1.455 ms.  The trio and pair kernels are candidates up to
// 2^16 txs (beyond that the one-lane kernel's throughput wins at any rounding).  secp256k1 recovery also
// has the row kernel (ecc_row.hip, one signature per workgroup): its first round of one signature per
// CU costs kRowLat of the trio's round and each further round kRowLatN (two workgroups share a CU:
// tools/small_sweep.py, profiles/r05_small_sweep_row.json: 0.127 / 0.153 / 0.211 / 0.280 / 0.347 ms at
// 1 / 256 / 512 / 768 / 1024 signatures against the trio's 0.378); SM2 its own row kernel, at
// kRowLatSM2 for one signature per CU and kRowLatNSM2 per further one while kRowResidentSM2 workgroups
// share a CU, a new round beyond (same file: 0.221 / 0.250 / 0.384 / 0.401 / 0.485 / 0.754 ms at 1 / 256 /
// 512 / 768 / 1024 / 1280 signatures against the trio's 0.578).
// Returns 3 (row), 2 (trio), 1 (pair), 0 (one-lane, occupancy 1) or -2 (one-lane, occupancy 2).
static constexpr double kRowLat = 0.38, kRowLatN = 0.18;
static constexpr double kRowLatSM2 = 0.43, kRowLatNSM2 = 0.14;
static constexpr uint64_t kRowResidentSM2 = 4;
static int auto_kernel(int suite, uint64_t n, int cus, bool small_ok, bool row_ok) {
    const bool sm2 = suite == BCOSGPU_SUITE_SM2;
    //                    occ 2,              occ 1,              pair,               trio
    const double lat[4] = {sm2 ? 4.315 : 4.475, sm2 ? 2.399 : 2.643, sm2 ? 1.678 : 1.279, 1.0};
    const double occ2_tail = sm2 ? 2.452 : 2.556;  // the occupancy-2 kernel's round of <= one wave per SIMD
    const uint64_t per[4] = {512ull * cus, 256ull * cus, 64ull * cus, 40ull * cus};
    const int code[4] = {-2, 0, 1, 2};
    int best = 0;
    double cost = 1e300;
    for (int k = small_ok ? 3 : 1; k >= 0; --k) {
        double c = static_cast<double>((n + per[k] - 1) / per[k]) * lat[k];
        if (k == 0) {  // occupancy 2: full rounds, then a tail round
            const uint64_t tail = n % per[0];
            c = static_cast<double>(n / per[0]) * lat[0] + (tail == 0 ? 0.0 : tail <= per[1] ? occ2_tail : lat[0]);
        }
        if (c < cost) {
            cost = c;
            best = code[k];
        }
    }
    if (row_ok && small_ok) {
        // m signatures per CU; a round holds `res` of them per CU (secp256k1: linear in m throughout)
        const double r1 = sm2 ? kRowLatSM2 : kRowLat, rn = sm2 ? kRowLatNSM2 : kRowLatN;
        const uint64_t m = (n + cus - 1) / cus, res = sm2 ? kRowResidentSM2 : m;
        const uint64_t rounds = (m + res - 1) / res;
        const double c = static_cast<double>(rounds) * r1 + static_cast<double>(m - rounds) * rn;
        if (c < cost) best = 3;
    }
    return best;
}

template <class IO>
int launch_verify(int suite, const IO& io, uint64_t n, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    TxKernelPolicy pol = tx_policy();
    constexpr bool kTx = std::is_same_v<IO, TxIO>;
    // small batches (SIMDs left idle by one tx per lane): the cooperative kernels -- secp256k1 in
    // ecc_coop.hip, SM2 in ecc_pair.hip -- chosen by rounds x latency when the policy is automatic
    bool small = pol.split >= 0 ? pol.split == 1 : n <= (1ull << 15);
    int occ = pol.occ;
    if (pol.split < 0 && pol.coop == 2 && pol.f26) {
        // the row kernels: secp256k1 recovery (TxIO, SigIO, EcrecIO; its known-key verify is chosen in
        // ecc_sig.hip) and SM2 verification (TxIO, SigIO, KeyIO); BCOSGPU_TXV_ROW=0 leaves them out
        static const bool row_env = [] {
            const char* e = getenv("BCOSGPU_TXV_ROW");
            return !(e && atoi(e) == 0);
        }();
        const bool row_io = suite == BCOSGPU_SUITE_SM2 || !std::is_same_v<IO, KeyIO>;
        const int k = auto_kernel(suite, n, cu_count(), n <= (1ull << 16), row_env && row_io);
        small = k > 0;
        if (small) pol.coop = k;
        else if (!occ) occ = k == -2 ? 2 : 1;
    }
    if (!occ) occ = n >= (1ull << 17) ? 2 : 1;  // forced non-automatic policies: >= 2 waves per SIMD of work
    // SigIO has the fe26 / fp26 cooperative kernels only; other policies take the one-lane kernel
    if (small && !kTx && !(pol.f26 && pol.coop)) small = false;
    // EcrecIO is a secp256k1 recovery only, KeyIO (here) an SM2 verification only
    constexpr bool kK1 = !std::is_same_v<IO, KeyIO>, kSM2 = !std::is_same_v<IO, EcrecIO>;
    if constexpr (kK1)
        if (suite == BCOSGPU_SUITE_SECP256K1 && small) return launch_verify_small_secp(pol, io, n, st);
    if constexpr (kSM2)
        if (suite == BCOSGPU_SUITE_SM2 && small && pol.coop) return launch_verify_small_sm2(pol, io, n, st);
#define TXV(S, O, F, T) \
    hipLaunchKernelGGL((tx_verify_kernel<S, O, F, IO>), dim3(grid_of(n)), dim3(256), 0, st, io, n, T, bits)
    if (suite == BCOSGPU_SUITE_SM2) {
        if constexpr (kSM2) {
            if (pol.f26) {
                const uint32_t* t26;
                rc = tables_sm2_26(&t26, &bits);
                if (rc) return rc;
                if (occ == 2) TXV(BCOSGPU_SUITE_SM2, 2, true, t26); else TXV(BCOSGPU_SUITE_SM2, 1, true, t26);
            } else {
                if (occ == 2 && kTx) TXV(BCOSGPU_SUITE_SM2, 2, false, sm2); else TXV(BCOSGPU_SUITE_SM2, 1, false, sm2);
            }
        } else {
            return BCOSGPU_E_ARG;
        }
    } else if constexpr (kK1) {
        if (pol.f26) {
            if (occ == 2) TXV(BCOSGPU_SUITE_SECP256K1, 2, true, k1); else TXV(BCOSGPU_SUITE_SECP256K1, 1, true, k1);
        } else {
            if (occ == 2 && kTx) TXV(BCOSGPU_SUITE_SECP256K1, 2, false, k1); else TXV(BCOSGPU_SUITE_SECP256K1, 1, false, k1);
        }
    } else {
        return BCOSGPU_E_ARG;
    }
#undef TXV
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_tx_verify(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off, const uint8_t* d_sig,
                     const uint64_t* d_sig_off, uint64_t n, uint8_t* d_txhash, uint8_t* d_sender, uint8_t* d_status,
                     hipStream_t st) {
    const TxIO io{d_pre, d_pre_off, d_sig, d_sig_off, d_txhash, d_sender, d_status};
    return launch_verify(suite, io, n, st);
}

// SignatureCrypto::recover (Secp256k1Crypto.cpp:79-93) for a batch: signature i = 65 bytes at
// d_sig + stride i; pub / addr nullable; ok = 1 / 0.
int launch_secp256k1_recover(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride, uint64_t n, uint8_t* d_pub,
                             uint8_t* d_addr, uint8_t* d_ok, hipStream_t st) {
    const SigIO io{d_hash, d_sig, stride, 65u, d_pub, d_addr, d_ok};
    return launch_verify(BCOSGPU_SUITE_SECP256K1, io, n, st);
}

// SM2Crypto::recover (SM2Crypto.cpp:81-92: verify against the embedded key) for a batch: signature i =
// r || s || pub (128 bytes) at d_sig + stride i; addr nullable; ok = 1 / 0.
int launch_sm2_verify(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride, uint64_t n, uint8_t* d_addr,
                      uint8_t* d_ok, hipStream_t st) {
    const SigIO io{d_hash, d_sig, stride, 128u, nullptr, d_addr, d_ok};
    return launch_verify(BCOSGPU_SUITE_SM2, io, n, st);
}

// The EVM ecRecover precompile (Precompiled.cpp:443-482) for a batch: the recovery kernels over EcrecIO,
// with the same rounds x latency choice (the lane-trio kernel for a block's few calls).
int launch_ecrecover(const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint8_t* d_ok, hipStream_t st) {
    const EcrecIO io{d_in, d_out, d_ok};
    return launch_verify(BCOSGPU_SUITE_SECP256K1, io, n, st);
}

// SignatureCrypto::verify with a known key, SM2 (SM2Crypto.cpp:66-79): the SM2 verification kernels over
// KeyIO, the key from pub64 instead of the signature's tail (ecc_sig.hip launch_sig_verify).
int launch_sm2_verify_key(const uint8_t* d_pub, const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride,
                          uint64_t n, uint8_t* d_ok, hipStream_t st) {
    const KeyIO io{d_pub, d_hash, d_sig, stride, d_ok};
    return launch_verify(BCOSGPU_SUITE_SM2, io, n, st);
}
}  // namespace bcosgpu
