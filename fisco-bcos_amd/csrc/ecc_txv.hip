// ecc_txv.hip -- the one-lane fused tx-admission kernel tx_verify_kernel<suite, occupancy, field> and
// launch_tx_verify, which routes small batches to the cooperative kernels (ecc_coop.hip, ecc_pair.hip).
#include "ecc_device.h"

namespace bcosgpu {

// Transaction::verify for a batch: tx hash of the preimage, recover / verify, sender address.
// OCC = waves per SIMD the register allocation must allow: 1 (no spills, lowest per-tx latency:
// small batches) or 2 (spills ~120 VGPRs to scratch but doubles the resident waves: large batches).
template <int SUITE, int OCC, bool F26 = false>
__global__ __launch_bounds__(256, OCC) void tx_verify_kernel(const uint8_t* __restrict__ pre,
                                                        const uint64_t* __restrict__ pre_off,
                                                        const uint8_t* __restrict__ sig,
                                                        const uint64_t* __restrict__ sig_off, uint64_t n,
                                                        const uint32_t* __restrict__ tab, int tbits,
                                                        uint8_t* __restrict__ txhash, uint8_t* __restrict__ sender,
                                                        uint8_t* __restrict__ status) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = pre_off[i], b = pre_off[i + 1];
    const uint32_t len = static_cast<uint32_t>(b - a);
    ByteReader rd(pre + a, len);
    uint32_t d[8];
    if (SUITE == BCOSGPU_SUITE_SM2) sm3_msg(rd, len, d);
    else keccak256_msg(rd, len, d);
    store_digest(SUITE == BCOSGPU_SUITE_SM2 ? SM3 : KECCAK256, txhash + 32 * i, d);
    fe h;
    if (SUITE == BCOSGPU_SUITE_SM2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) h.v[k] = d[7 - k];
    } else {
        fe_from_be_words(h, d);
    }
    const uint64_t sa = sig_off[i], sb = sig_off[i + 1];
    const uint64_t slen64 = sb - sa;
    const uint32_t slen = slen64 > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(slen64);
    fe x, y;
    uint32_t ad[5] = {0, 0, 0, 0, 0};
    bool ok;
    // OCC 2: the variable-base table's x-coordinates live in LDS (16 KiB per wave, 128 KiB per CU
    // at 2 workgroups per CU), the rest of the working set in 256 VGPRs
    constexpr bool kLds = OCC == 2;
    __shared__ uint32_t ldsx_all[kLds ? 4 * 4096 : 1];
    uint32_t* ldsx = kLds ? ldsx_all + (threadIdx.x >> 6) * 4096 + (threadIdx.x & 63) : nullptr;
    if (SUITE == BCOSGPU_SUITE_SM2) {
        if constexpr (F26) ok = sm2_verify_lane26<kLds>(h, sig + sa, slen, CombTab{tab, tbits}, x, y, ldsx);
        else ok = sm2_verify_lane<kLds>(h, sig + sa, slen, CombTab{tab, tbits}, x, y, ldsx);
        if (ok) sm3_address(ad, x, y);
    } else {
        if constexpr (F26) ok = secp256k1_recover_lane26<kLds>(h, sig + sa, slen, CombTab{tab, tbits}, x, y, ldsx);
        else ok = secp256k1_recover_lane<kLds>(h, sig + sa, slen, CombTab{tab, tbits}, x, y, ldsx);
        if (ok) keccak_address(ad, x, y);
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = ad[k];
    status[i] = ok ? 0 : 1;
}


// The automatic choice for batches up to 2^16 (policy split = -1, coop = 2, field = 1): each kernel
// runs its batch in rounds of resident workgroups -- the trio kernels take 40 txs per CU, the pair
// kernels 64, the one-lane kernel 256 (one wave per SIMD) -- and a round costs a fixed latency, so
// the cost is rounds x latency.  The latencies are relative to the trio kernel's, measured on MI355X
// (tools/small_sweep.py, profiles/r02_small_sweep.json: secp256k1 trio 0.415 / pair 0.493 / one-lane
// 0.98 ms per round; SM2 0.854 / 0.977 / 1.51).  Returns 2 (trio), 1 (pair) or 0 (one-lane).
static int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}
static int auto_small_kernel(int suite, uint64_t n, int cus) {
    const bool sm2 = suite == BCOSGPU_SUITE_SM2;
    const double lat[3] = {sm2 ? 1.77 : 2.36, sm2 ? 1.15 : 1.19, 1.0};  // one-lane, pair, trio
    const uint64_t per[3] = {256ull * cus, 64ull * cus, 40ull * cus};
    int best = 2;
    double cost = 1e30;
    for (int k = 2; k >= 0; --k) {
        const double c = static_cast<double>((n + per[k] - 1) / per[k]) * lat[k];
        if (c < cost) {
            cost = c;
            best = k;
        }
    }
    return best;
}

int launch_tx_verify(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off, const uint8_t* d_sig,
                     const uint64_t* d_sig_off, uint64_t n, uint8_t* d_txhash, uint8_t* d_sender, uint8_t* d_status,
                     hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    TxKernelPolicy pol = tx_policy();
    // small batches (SIMDs left idle by one tx per lane): the cooperative kernels -- secp256k1 (C2) in
    // ecc_coop.hip, SM2 in ecc_pair.hip -- chosen by rounds x latency when the policy is automatic
    bool small = pol.split >= 0 ? pol.split == 1 : n <= (1ull << 15);
    if (pol.split < 0 && pol.coop == 2 && pol.f26) {
        const int k = n <= (1ull << 16) ? auto_small_kernel(suite, n, cu_count()) : 0;
        small = k != 0;
        if (small) pol.coop = k;
    }
    if (suite == BCOSGPU_SUITE_SECP256K1 && small)
        return launch_tx_verify_small_secp(pol, d_pre, d_pre_off, d_sig, d_sig_off, n, d_txhash, d_sender, d_status, st);
    if (suite == BCOSGPU_SUITE_SM2 && small && pol.coop)
        return launch_tx_verify_small_sm2(pol, d_pre, d_pre_off, d_sig, d_sig_off, n, d_txhash, d_sender, d_status, st);
    const int occ = pol.occ ? pol.occ : (n >= (1ull << 17) ? 2 : 1);  // >= 2 waves per SIMD of work
#define TXV(S, O, F, T) hipLaunchKernelGGL((tx_verify_kernel<S, O, F>), dim3(grid_of(n)), dim3(256), 0, st, d_pre, \
                                           d_pre_off, d_sig, d_sig_off, n, T, bits, d_txhash, d_sender, d_status)
    if (suite == BCOSGPU_SUITE_SM2 && pol.f26) {
        const uint32_t* t26;
        rc = tables_sm2_26(&t26, &bits);
        if (rc) return rc;
        if (occ == 2) TXV(BCOSGPU_SUITE_SM2, 2, true, t26); else TXV(BCOSGPU_SUITE_SM2, 1, true, t26);
    } else if (suite == BCOSGPU_SUITE_SM2) {
        if (occ == 2) TXV(BCOSGPU_SUITE_SM2, 2, false, sm2); else TXV(BCOSGPU_SUITE_SM2, 1, false, sm2);
    } else if (pol.f26) {
        if (occ == 2) TXV(BCOSGPU_SUITE_SECP256K1, 2, true, k1); else TXV(BCOSGPU_SUITE_SECP256K1, 1, true, k1);
    } else {
        if (occ == 2) TXV(BCOSGPU_SUITE_SECP256K1, 2, false, k1); else TXV(BCOSGPU_SUITE_SECP256K1, 1, false, k1);
    }
#undef TXV
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
}  // namespace bcosgpu
