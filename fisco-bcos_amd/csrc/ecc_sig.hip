// ecc_sig.hip -- the one-lane known-key verify kernel and the deterministic signing used to build
// synthetic batches; the known-key verify launcher.  (Recover, SM2 verify with the digest given and the
// ecRecover precompile run the tx-verify kernels over SigIO / EcrecIO: ecc_txv.hip; the small-batch
// known-key verify runs on lane trios: ecc_coop.hip sig_verify_trio26_kernel, ecc_pair.hip over KeyIO.)
#include "ecc_device.h"

namespace bcosgpu {

// ------------------------------------------------------------------ kernels
// SignatureCrypto::verify(pub, hash, sig) for a batch (sealer signatures: BlockValidator.cpp:141-182,
// PBFTCacheProcessor.cpp:795-821).  SM2: SM2Crypto::verify reads the first 64 signature bytes (r || s)
// and verifies against the GIVEN key (SM2Crypto.cpp:66-79); secp256k1: secp256k1_verify_lane.
template <int SUITE, bool F26 = false>
__global__ __launch_bounds__(256) void sig_verify_kernel(const uint8_t* __restrict__ pub,
                                                         const uint8_t* __restrict__ hash,
                                                         const uint8_t* __restrict__ sig, uint32_t stride,
                                                         uint64_t n, const uint32_t* __restrict__ tab, int tbits,
                                                         uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe h;
    load_be256_aligned(h, hash + 32 * i);
    const uint8_t* sg = sig + static_cast<uint64_t>(stride) * i;
    bool ok;
    if (SUITE == BCOSGPU_SUITE_SM2) {
        ByteReader rs(sg, 64), rp(pub + 64 * i, 64);
        uint32_t w[8], X[8], Y[8];
        fe r, s, x, y;
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rs.word(k);
        fe_from_be_words(r, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rs.word(8 + k);
        fe_from_be_words(s, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            X[k] = bswap32(rp.word(k));
            Y[k] = bswap32(rp.word(8 + k));
        }
        if constexpr (F26) ok = sm2_verify_rs26(h, r, s, X, Y, CombTab{tab, tbits}, x, y);
        else ok = sm2_verify_rs(h, r, s, X, Y, CombTab{tab, tbits}, x, y);
    } else {
        if constexpr (F26) ok = secp256k1_verify_lane26(h, sg, pub + 64 * i, CombTab{tab, tbits});
        else ok = secp256k1_verify_lane(h, sg, pub + 64 * i, CombTab{tab, tbits});
    }
    okout[i] = ok ? 1 : 0;
}

// Key derivation + deterministic ECDSA signing, libsecp256k1 conventions (low-S, recid).
// k = Keccak256(sk || hash) mod n.
__global__ __launch_bounds__(256) void secp256k1_sign_kernel(const uint8_t* __restrict__ sk32,
                                                             const uint8_t* __restrict__ hash32, uint64_t n,
                                                             const uint32_t* __restrict__ tab, int tbits,
                                                             uint8_t* __restrict__ pub, uint8_t* __restrict__ sigout,
                                                             uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* skw = reinterpret_cast<const uint4*>(sk32 + 32 * i);
    const uint4* hw = reinterpret_cast<const uint4*>(hash32 + 32 * i);
    const uint4 s0 = skw[0], s1 = skw[1], h0 = hw[0], h1 = hw[1];
    const uint32_t m[16] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w,
                            h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    fe d, e, k;
    fe_from_be_words(d, m);
    fe_from_be_words(e, m + 8);
    uint32_t kd[8];
    keccak256_64(m, kd);
    fe_from_be_words(k, kd);
    reduce_once(k, ParamN1::M);
    reduce_once(e, ParamN1::M);
    bool ok = !fe_is_zero_raw(d) && fe_lt_k(d, ParamN1::M) && !fe_is_zero_raw(k);
    Jac P, R;
    Aff PA, RA;
    comb_mul_rt<CurveK1>(P, d, tab, tbits);
    comb_mul_rt<CurveK1>(R, k, tab, tbits);
    CurveK1::to_aff(PA, P);
    CurveK1::to_aff(RA, R);
    FieldK1::normalize(PA.x);
    FieldK1::normalize(PA.y);
    FieldK1::normalize(RA.x);
    FieldK1::normalize(RA.y);
    uint32_t recid = RA.y.v[0] & 1u;
    fe r;
    fe_copy(r, RA.x);
    if (!fe_lt_k(r, ParamN1::M)) recid |= 2u;
    reduce_once(r, ParamN1::M);
    ok = ok && !fe_is_zero_raw(r);
    // s = k^-1 (e + r d) mod n
    fe km, kinv, dm, rd, t, s;
    fe kk = k;
    if (fe_is_zero_raw(kk)) kk.v[0] = 1;
    FieldN1::from_plain(km, kk);
    FieldInv<FieldN1>::inv(kinv, km);
    FieldN1::from_plain(dm, d);
    FieldN1::mul(rd, r, dm);
    FieldN1::add(t, e, rd);
    FieldN1::mul(s, t, kinv);
    ok = ok && !fe_is_zero_raw(s);
    fe half;
    fe_set(half, kN1Half);
    if (fe_lt(half, s)) {
        FieldN1::neg(s, s);
        recid ^= 1u;
    }
    store_be256(pub + 64 * i, PA.x);
    store_be256(pub + 64 * i + 32, PA.y);
    uint8_t* so = sigout + 65 * i;
    uint32_t rw[8], sw[8];
    fe_to_be_words(rw, r);
    fe_to_be_words(sw, s);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
        so[q] = static_cast<uint8_t>(rw[q >> 2] >> ((q & 3) * 8));
        so[32 + q] = static_cast<uint8_t>(sw[q >> 2] >> ((q & 3) * 8));
    }
    so[64] = static_cast<uint8_t>(recid);
    okout[i] = ok ? 1 : 0;
}

// SM2 key derivation + signing (GB/T 32918.2), k = SM3(sk || hash) mod n; sig = r || s || pub.
__global__ __launch_bounds__(256) void sm2_sign_kernel(const uint8_t* __restrict__ sk32,
                                                       const uint8_t* __restrict__ hash32, uint64_t n,
                                                       const uint32_t* __restrict__ tab, int tbits,
                                                       uint8_t* __restrict__ sigout, uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe d, h;
    load_be256_aligned(d, sk32 + 32 * i);
    load_be256_aligned(h, hash32 + 32 * i);
    // k = SM3(sk || hash)
    uint32_t W[16], V[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        W[j] = d.v[7 - j];
        W[8 + j] = h.v[7 - j];
    }
    sm3_init(V);
    sm3_compress(V, W);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = 0;
    W[0] = 0x80000000u;
    W[15] = 512u;
    sm3_compress(V, W);
    fe k;
#pragma unroll
    for (int j = 0; j < 8; ++j) k.v[j] = V[7 - j];
    reduce_once(k, ParamN2::M);
    fe nm1;
    fe_set(nm1, ParamN2::M);
    nm1.v[0] -= 1;  // n - 1 (low limb of n is odd and > 0)
    bool ok = !fe_is_zero_raw(d) && fe_lt(d, nm1) && !fe_is_zero_raw(k);
    Jac P, K;
    Aff PA, KA;
    comb_mul_rt<CurveSM2>(P, d, tab, tbits);
    comb_mul_rt<CurveSM2>(K, k, tab, tbits);
    CurveSM2::to_aff(PA, P);
    CurveSM2::to_aff(KA, K);
    fe px, py, x1;
    FieldP2::to_plain(px, PA.x);
    FieldP2::to_plain(py, PA.y);
    FieldP2::to_plain(x1, KA.x);
    uint32_t X[8], Y[8], eb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        X[j] = px.v[7 - j];
        Y[j] = py.v[7 - j];
    }
    sm2_e(eb, X, Y, h);
    fe e;
#pragma unroll
    for (int j = 0; j < 8; ++j) e.v[j] = eb[7 - j];
    reduce_once(e, ParamN2::M);
    reduce_once(x1, ParamN2::M);
    fe r, t, s;
    FieldN2::add(r, e, x1);
    ok = ok && !fe_is_zero_raw(r);
    FieldN2::add(t, r, k);
    ok = ok && !fe_is_zero_raw(t);
    fe one, dp1, dm, inv, rd;
    fe_zero(one);
    one.v[0] = 1;
    FieldN2::add(dp1, d, one);
    if (fe_is_zero_raw(dp1)) dp1.v[0] = 1;
    FieldN2::from_plain(dm, dp1);
    FieldInv<FieldN2>::inv(inv, dm);
    fe dmm;
    FieldN2::from_plain(dmm, d);
    FieldN2::mul(rd, r, dmm);
    FieldN2::sub(t, k, rd);
    FieldN2::mul(s, t, inv);
    ok = ok && !fe_is_zero_raw(s);
    uint8_t* so = sigout + 128 * i;
    uint32_t w[8];
    const fe* parts[4] = {&r, &s, &px, &py};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        fe_to_be_words(w, *parts[p]);
#pragma unroll
        for (int q = 0; q < 8; ++q) reinterpret_cast<uint32_t*>(so + 32 * p)[q] = w[q];
    }
    okout[i] = ok ? 1 : 0;
}

// Signing exists to build the synthetic benchmark / test batches on the device.  It is NOT
// constant-time (the comb gather address depends on secret key and nonce bits): test use only.
int launch_secp256k1_sign(const uint8_t* d_sk, const uint8_t* d_hash, uint64_t n, uint8_t* d_pub, uint8_t* d_sig,
                          uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    if (!d_pub) return BCOSGPU_E_ARG;
    hipLaunchKernelGGL(secp256k1_sign_kernel, dim3(grid_of(n)), dim3(256), 0, st, d_sk, d_hash, n, k1, bits, d_pub,
                       d_sig, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_sm2_sign(const uint8_t* d_sk, const uint8_t* d_hash, uint64_t n, uint8_t* d_sig, uint8_t* d_ok,
                    hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL(sm2_sign_kernel, dim3(grid_of(n)), dim3(256), 0, st, d_sk, d_hash, n, sm2, bits, d_sig, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

// The known-key verify batch (bcosgpu_verify_batch*): SM2 runs the SM2 verification kernels over KeyIO
// (the same rounds x latency choice as recover / tx verify, ecc_txv.hip launch_sm2_verify_key);
// secp256k1 runs the lane-trio verify kernel for batches of up to two trio rounds (a block's sealer
// signatures: the latency path) and the one-lane sig_verify_kernel beyond (the trio kernel's round is
// ~3x shorter than the one-lane kernel's, which fits 6.4x more signatures per round: tools/small_sweep.py
// verify, profiles/r04_verify_sweep.json).  Policy split 1 / 0 forces the trio / one-lane kernel.
// the row verify kernel's rounds of one signature per CU: 0.104 / 0.131 / 0.169 / 0.217 ms at 1 / 256 /
// 512 / 768 signatures against the trio's 0.338 (profiles/r05_verify_sweep_row.json)
static constexpr uint64_t kRowVerifyRounds = 4;
int launch_sig_verify(int suite, const uint8_t* d_pub, const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride,
                      uint64_t n, uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    const TxKernelPolicy pol = tx_policy();
    if (suite == BCOSGPU_SUITE_SM2 && pol.f26) return launch_sm2_verify_key(d_pub, d_hash, d_sig, stride, n, d_ok, st);
    if (suite == BCOSGPU_SUITE_SECP256K1 && pol.f26 && pol.coop >= 2) {
        const uint64_t cus = static_cast<uint64_t>(cu_count());
        const bool small = pol.split >= 0 ? pol.split == 1 : n <= 2ull * 40 * cus;
        // the row kernel (ecc_row.hip) while its rounds of one signature per CU beat the trio's round
        // (tools/small_sweep.py verify, profiles/r05_verify_sweep_row.json); coop 3 forces it
        static const bool row_env = [] {
            const char* e = getenv("BCOSGPU_TXV_ROW");
            return !(e && atoi(e) == 0);
        }();
        const bool row = pol.coop == 3 || (pol.split < 0 && row_env && n <= kRowVerifyRounds * cus);
        if (small && row) return launch_sig_verify_row_secp(KeyIO{d_pub, d_hash, d_sig, stride, d_ok}, n, st);
        if (small) return launch_sig_verify_small_secp(KeyIO{d_pub, d_hash, d_sig, stride, d_ok}, n, st);
    }
    if (suite == BCOSGPU_SUITE_SM2)
        hipLaunchKernelGGL(sig_verify_kernel<BCOSGPU_SUITE_SM2>, dim3(grid_of(n)), dim3(256), 0, st, d_pub, d_hash, d_sig,
                           stride, n, sm2, bits, d_ok);
    else if (pol.f26)
        hipLaunchKernelGGL((sig_verify_kernel<BCOSGPU_SUITE_SECP256K1, true>), dim3(grid_of(n)), dim3(256), 0, st, d_pub,
                           d_hash, d_sig, stride, n, k1, bits, d_ok);
    else
        hipLaunchKernelGGL(sig_verify_kernel<BCOSGPU_SUITE_SECP256K1>, dim3(grid_of(n)), dim3(256), 0, st, d_pub, d_hash,
                           d_sig, stride, n, k1, bits, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

}  // namespace bcosgpu
