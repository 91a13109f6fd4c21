// ecc_kernels.hip -- secp256k1 public-key recovery, SM2 verification, deterministic signing and the
// fused tx-admission kernel (gfx950, one signature per lane, integer ALU only).
//
// Replaces (per item, batched):
//   Secp256k1Crypto::recover -> wedpr_secp256k1_recover_public_key
//       bcos-crypto/bcos-crypto/signature/secp256k1/Secp256k1Crypto.cpp:79-93 (libsecp256k1 semantics)
//   SM2Crypto::recover -> verify -> fast_sm2_verify / sm2_do_verify
//       bcos-crypto/bcos-crypto/signature/sm2/SM2Crypto.cpp:66-92, fastsm2/fast_sm2.cpp:139-227
//   Transaction::verify (hash -> recover -> right160(H(pub)))
//       bcos-framework/bcos-framework/protocol/Transaction.h:68-82
//
// Scalar multiplication:
//   fixed base G : 8-bit comb, table[32][256] of affine multiples b*2^(8i)*G in HBM (512 KiB per
//                  curve, L2-resident), 32 mixed additions and no doublings.
//   variable base: radix-16 Booth recoding (digits in [-8, 8]) over a register-resident table of
//                  1P..8P; every lane runs the same 65-window schedule (no divergence).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include "ec.h"
#include "engine.h"
#include "hash_device.h"

namespace bcosgpu {

// ------------------------------------------------------------------ curve constants (internal form)
__device__ __constant__ static const uint32_t kK1Gx[8] = {0x16f81798u, 0x59f2815bu, 0x2dce28d9u, 0x029bfcdbu,
                                                       0xce870b07u, 0x55a06295u, 0xf9dcbbacu, 0x79be667eu};
__device__ __constant__ static const uint32_t kK1Gy[8] = {0xfb10d4b8u, 0x9c47d08fu, 0xa6855419u, 0xfd17b448u,
                                                       0x0e1108a8u, 0x5da4fbfcu, 0x26a3c465u, 0x483ada77u};
// p - n (recid & 2 requires r < p - n)
__device__ __constant__ static const uint32_t kK1PminusN[8] = {0x2fc9baeeu, 0x402da172u, 0x50b75fc4u, 0x45512319u,
                                                            0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u};
__device__ __constant__ static const uint32_t kN1Half[8] = {0x681b20a0u, 0xdfe92f46u, 0x57a4501du, 0x5d576e73u,
                                                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
// GLV endomorphism of secp256k1: lambda*(x, y) = (beta*x, y); split constants of libsecp256k1's
// secp256k1_scalar_split_lambda (|k1|, |k2| < 2^128).  LAMBDA and MINUS_B2 in Montgomery form mod n.
__device__ __constant__ static const uint32_t kGlvG1[8] = {0x45dbb031u, 0xe893209au, 0x71e8ca7fu, 0x3daa8a14u,
                                                        0x9284eb15u, 0xe86c90e4u, 0xa7d46bcdu, 0x3086d221u};
__device__ __constant__ static const uint32_t kGlvG2[8] = {0x8ac47f71u, 0x1571b4aeu, 0x9df506c6u, 0x221208acu,
                                                        0x0abfe4c4u, 0x6f547fa9u, 0x010e8828u, 0xe4437ed6u};
__device__ __constant__ static const uint32_t kGlvMB1[8] = {0x0abfe4c3u, 0x6f547fa9u, 0x010e8828u, 0xe4437ed6u,
                                                         0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u};
__device__ __constant__ static const uint32_t kGlvMB2M[8] = {0x6a144696u, 0x0cac5e50u, 0xf3ba5939u, 0x1e8a8dc5u,
                                                          0xba244fceu, 0x176cdf65u, 0x8e173580u, 0xc25575ebu};
__device__ __constant__ static const uint32_t kGlvLambdaM[8] = {0xc9926c9eu, 0xf07deb3du, 0x83c6944cu, 0x2c93e7adu,
                                                             0x52697d91u, 0x73a96606u, 0x8558d639u, 0x53284017u};
__device__ __constant__ static const uint32_t kGlvBeta[8] = {0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u,
                                                          0xac3434e9u, 0x6e64479eu, 0x657c0710u, 0x7ae96a2bu};
// SM2 (Montgomery form mod p)
__device__ __constant__ static const uint32_t kSM2Gx[8] = {0xf418029eu, 0x61328990u, 0xdca6c050u, 0x3e7981edu,
                                                        0xac24c3c3u, 0xd6a1ed99u, 0xe1c13b05u, 0x91167a5eu};
__device__ __constant__ static const uint32_t kSM2Gy[8] = {0x3c2d0dddu, 0xc1354e59u, 0x8d3295fau, 0xc1f5e578u,
                                                        0x6e2a48f8u, 0x8d4cfb06u, 0x81d735bdu, 0x63cd65d4u};
__device__ __constant__ static const uint32_t kSM2B[8] = {0x2bc0dd42u, 0x90d23063u, 0xe9b537abu, 0x71cf379au,
                                                       0x5ea51c3cu, 0x52798150u, 0xba20e2c8u, 0x240fe188u};
// Z_A = SM3(ENTL || "1234567812345678" || a || b || xG || yG || xA || yA) (fast_sm2.cpp:34,203):
// SM3 state after the key-independent first 128 bytes, the next 4 constant words and bytes 144..145.
__device__ __constant__ static const uint32_t kZaMid[8] = {0xadadedb5u, 0x0446043fu, 0x08a87aceu, 0xe86d2243u,
                                                        0x8e232383u, 0xbfc81fe2u, 0xcf9117c8u, 0x4707011du};
__device__ __constant__ static const uint32_t kZaW32[4] = {0x2153d0a9u, 0x877cc62au, 0x474002dfu, 0x32e52139u};
static constexpr uint32_t kZaC36 = 0xf0a00000u;

// ------------------------------------------------------------------ per-device G tables
// Two comb tables of affine b * 2^(B i) * G per curve, [window i][entry b][x0..7, y0..7]:
//  * 8-bit  (B = 8, 32 windows x 256, 512 KiB): L2-resident; the latency-bound small-batch kernels
//    (cooperative / split), whose lone waves would stall on every HBM gather;
//  * 16-bit (B = 16, 16 windows x 65536, 64 MiB): half the mixed additions (16 instead of 32) for
//    the throughput kernels, which hide the gather latency (one window prefetched, 2 waves/SIMD).
static constexpr int kCombWindows = 32;
static constexpr int kCombEntries = 256;
static constexpr size_t kTabWords = static_cast<size_t>(kCombWindows) * kCombEntries * 16;
static constexpr int kWideBits = 16;
static constexpr int kWideWindows = 256 / kWideBits;
static constexpr uint32_t kWideEntries = 1u << kWideBits;
static constexpr size_t kWideTabWords = static_cast<size_t>(kWideWindows) * kWideEntries * 16;
static std::mutex g_tab_mu;
static uint32_t* g_tab_k1[64];
static uint32_t* g_tab_sm2[64];
static uint32_t* g_wtab_k1[64];
static uint32_t* g_wtab_sm2[64];
static uint32_t* g_tab_sm2_26[64];   // the SM2 tables re-expressed in fp26's Montgomery domain (R = 2^286)
static uint32_t* g_wtab_sm2_26[64];

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ void load_be256(fe& r, const uint8_t* p) {
    ByteReader rd(p, 32);
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(i);
    fe_from_be_words(r, w);
}
__device__ __forceinline__ void load_be256_aligned(fe& r, const uint8_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    fe_from_be_words(r, w);
}
__device__ __forceinline__ void store_be256(uint8_t* p, const fe& a) {
    uint32_t w[8];
    fe_to_be_words(w, a);
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
__device__ __forceinline__ void store_be256_u32(uint8_t* p, const fe& a) {
    uint32_t w[8];
    fe_to_be_words(w, a);
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = w[i];
}
__device__ __forceinline__ void shr8(fe& k) {
#pragma unroll
    for (int i = 0; i < 7; ++i) k.v[i] = __builtin_amdgcn_alignbit(k.v[i + 1], k.v[i], 8);
    k.v[7] >>= 8;
}
__device__ __forceinline__ void shl4(fe& k) {
#pragma unroll
    for (int i = 7; i > 0; --i) k.v[i] = __builtin_amdgcn_alignbit(k.v[i], k.v[i - 1], 28);
    k.v[0] <<= 4;
}
__device__ __forceinline__ void shl1(fe& k) {
#pragma unroll
    for (int i = 7; i > 0; --i) k.v[i] = __builtin_amdgcn_alignbit(k.v[i], k.v[i - 1], 31);
    k.v[0] <<= 1;
}
// x mod n for x < 2^256 (n > 2^255)
__device__ __forceinline__ void reduce_once(fe& x, const uint32_t* n) {
    fe t;
    const uint32_t bw = fe_sub_k(t, x, n);
    fe_cmov(x, t, bw == 0);
}

// ------------------------------------------------------------------ scalar multiplication
template <int BITS>
__device__ __forceinline__ void shr_bits(fe& k) {
#pragma unroll
    for (int i = 0; i < 7; ++i) k.v[i] = __builtin_amdgcn_alignbit(k.v[i + 1], k.v[i], BITS);
    k.v[7] >>= BITS;
}
__device__ __forceinline__ void load_aff16(Aff& T, const uint32_t* __restrict__ e32) {
    const uint4* e = reinterpret_cast<const uint4*>(e32);
    const uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
    T.x.v[0] = q0.x; T.x.v[1] = q0.y; T.x.v[2] = q0.z; T.x.v[3] = q0.w;
    T.x.v[4] = q1.x; T.x.v[5] = q1.y; T.x.v[6] = q1.z; T.x.v[7] = q1.w;
    T.y.v[0] = q2.x; T.y.v[1] = q2.y; T.y.v[2] = q2.z; T.y.v[3] = q2.w;
    T.y.v[4] = q3.x; T.y.v[5] = q3.y; T.y.v[6] = q3.z; T.y.v[7] = q3.w;
}

// acc = k * G via a BITS-bit comb table (k plain, < 2^256): 256 / BITS mixed additions, no
// doublings.  The entry of window i + 1 is gathered before the addition of window i.
template <class C, int BITS = kWideBits>
__device__ __forceinline__ void comb_mul(Jac& acc, const fe& k_plain, const uint32_t* __restrict__ tab) {
    constexpr int W = 256 / BITS;
    constexpr uint32_t E = 1u << BITS, MASK = E - 1u;
    fe k;
    fe_copy(k, k_plain);
    C::set_inf(acc);
    uint32_t b = k.v[0] & MASK;
    shr_bits<BITS>(k);
    Aff T;
    load_aff16(T, tab + static_cast<size_t>(b) * 16);
#pragma unroll 1
    for (int i = 0; i < W; ++i) {
        const uint32_t bi = b;
        Aff N;
        const int in = i + 1 < W ? i + 1 : i;  // last window: a harmless reload
        b = k.v[0] & MASK;
        shr_bits<BITS>(k);
        load_aff16(N, tab + (static_cast<size_t>(in) * E + b) * 16);
        Jac S;
        C::madd(S, acc, T);
        C::cmov(acc, S, bi != 0u);
        fe_copy(T.x, N.x);
        fe_copy(T.y, N.y);
    }
}

struct CombTab {
    const uint32_t* p;
    int bits;
};

// comb_mul over whichever table the device holds: the 16-bit one, or the 8-bit one when the 64 MiB
// tables were not allocated (bcosgpu_init_ex flag / allocation failure); tbits is launch-uniform
template <class C>
__device__ __forceinline__ void comb_mul_rt(Jac& acc, const fe& k, const uint32_t* __restrict__ tab, int tbits) {
    if (tbits == kWideBits) comb_mul<C, kWideBits>(acc, k, tab);
    else comb_mul<C, 8>(acc, k, tab);
}

// acc = k * P, radix-16 Booth recoding over the table 1P..8P (k plain, < 2^256)
template <class C, class F>
__device__ __forceinline__ void booth_mul(Jac& acc, const fe& k_plain, const Aff& P) {
    Jac T[8];
    C::from_aff(T[0], P);
    C::dbl(T[1], T[0]);
    C::madd(T[2], T[1], P);
    C::dbl(T[3], T[1]);
    C::madd(T[4], T[3], P);
    C::dbl(T[5], T[2]);
    C::madd(T[6], T[5], P);
    C::dbl(T[7], T[3]);
    fe k;
    fe_copy(k, k_plain);
    C::set_inf(acc);
    C::cmov(acc, T[0], (k.v[7] >> 31) != 0u);  // digit 64 = bit 255
#pragma unroll 1
    for (int i = 63; i >= 0; --i) {
        C::dbl(acc, acc);
        C::dbl(acc, acc);
        C::dbl(acc, acc);
        C::dbl(acc, acc);
        const uint32_t top = k.v[7];
        const uint32_t W = top >> 28, c = (top >> 27) & 1u;
        const int d = static_cast<int>(W + c) - static_cast<int>((W >> 3) << 4);
        shl4(k);
        const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
        Jac S;
        fe_copy(S.X, T[0].X); fe_copy(S.Y, T[0].Y); fe_copy(S.Z, T[0].Z); S.inf = false;
#pragma unroll
        for (int q = 1; q < 8; ++q) {
            const bool take = m == static_cast<uint32_t>(q);
            fe_cmov(S.X, T[q].X, take);
            fe_cmov(S.Y, T[q].Y, take);
            fe_cmov(S.Z, T[q].Z, take);
        }
        fe ny;
        F::neg(ny, S.Y);
        fe_cmov(S.Y, ny, d < 0);
        Jac R;
        C::add(R, acc, S);
        C::cmov(acc, R, d != 0);
    }
}

// k = k1 + k2*lambda (mod n) with |k1|, |k2| < 2^128 (libsecp256k1 split_lambda); returns the
// magnitudes and signs.
__device__ __forceinline__ void glv_split(fe& k1, bool& neg1, fe& k2, bool& neg2, const fe& k) {
    uint32_t t[16];
    fe g, c1, c2, x, y;
    fe_set(g, kGlvG1);
    mul_512(t, k, g);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) c1.v[i] = addc32(t[12 + i], i == 0 ? (t[11] >> 31) : 0u, c, c);
#pragma unroll
    for (int i = 4; i < 8; ++i) c1.v[i] = 0;
    fe_set(g, kGlvG2);
    mul_512(t, k, g);
    c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) c2.v[i] = addc32(t[12 + i], i == 0 ? (t[11] >> 31) : 0u, c, c);
#pragma unroll
    for (int i = 4; i < 8; ++i) c2.v[i] = 0;
    fe_set(g, kGlvMB1);
    mul_512(t, c1, g);  // < 2^256
#pragma unroll
    for (int i = 0; i < 8; ++i) x.v[i] = t[i];
    reduce_once(x, ParamN1::M);
    fe_set(g, kGlvMB2M);
    FieldN1::mul(y, c2, g);  // c2 * (-b2) mod n
    FieldN1::add(k2, x, y);
    fe_set(g, kGlvLambdaM);
    FieldN1::mul(x, k2, g);  // k2 * lambda mod n
    FieldN1::sub(k1, k, x);
    fe half, nk;
    fe_set(half, kN1Half);
    neg1 = fe_lt(half, k1);
    FieldN1::neg(nk, k1);
    fe_cmov(k1, nk, neg1);
    neg2 = fe_lt(half, k2);
    FieldN1::neg(nk, k2);
    fe_cmov(k2, nk, neg2);
}

__device__ __forceinline__ void shl4_128(fe& k) {
#pragma unroll
    for (int i = 3; i > 0; --i) k.v[i] = __builtin_amdgcn_alignbit(k.v[i], k.v[i - 1], 28);
    k.v[0] <<= 4;
}

// one Booth digit of a 128-bit scalar held in k.v[0..3], window at bits 124..127
__device__ __forceinline__ int booth_digit128(fe& k) {
    const uint32_t top = k.v[3];
    const uint32_t W = top >> 28, c = (top >> 27) & 1u;
    shl4_128(k);
    return static_cast<int>(W + c) - static_cast<int>((W >> 3) << 4);
}

// acc += (sign * d) * (phi ? lambda : 1) * P over an affine table T[j] = (j+1) P (mixed add)
template <class C, class F>
__device__ __forceinline__ void add_digit_aff(Jac& acc, const Aff T[8], int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    Aff S;
    fe_copy(S.x, T[0].x);
    fe_copy(S.y, T[0].y);
#pragma unroll
    for (int q = 1; q < 8; ++q) {
        const uint64_t take = __builtin_amdgcn_ballot_w64(m == static_cast<uint32_t>(q));
        fe_cmov_mask(S.x, T[q].x, take);
        fe_cmov_mask(S.y, T[q].y, take);
    }
    if (phi) {
        fe b;
        fe_set(b, kGlvBeta);
        F::mul(S.x, S.x, b);
    }
    fe ny;
    F::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    C::madd(R, acc, S);
    C::cmov(acc, R, d != 0);
}

// Same, with the table's x-coordinates in a per-wave LDS slice laid out [entry][word][lane] (a
// conflict-free per-lane gather of 8 dwords) and the y-coordinates in VGPRs: frees 64 VGPRs, so the
// occupancy-2 kernels stop spilling the table to scratch.
template <class C, class F>
__device__ __forceinline__ void add_digit_ldsx(Jac& acc, const uint32_t* ldsx, const fe Y[8], int d, bool neg,
                                               bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    Aff S;
    const uint32_t* b = ldsx + m * 512u;
#pragma unroll
    for (int k = 0; k < 8; ++k) S.x.v[k] = b[k * 64];
    fe_copy(S.y, Y[0]);
#pragma unroll
    for (int q = 1; q < 8; ++q) fe_cmov_mask(S.y, Y[q], __builtin_amdgcn_ballot_w64(m == static_cast<uint32_t>(q)));
    if (phi) {
        fe bt;
        fe_set(bt, kGlvBeta);
        F::mul(S.x, S.x, bt);
    }
    fe ny;
    F::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    C::madd(R, acc, S);
    C::cmov(acc, R, d != 0);
}

// Moves the table's x-coordinates to the wave's LDS slice (ldsx already offset by the lane).
__device__ __forceinline__ void table_x_to_lds(uint32_t* ldsx, const Aff A[8], fe Y[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int k = 0; k < 8; ++k) ldsx[(j * 8 + k) * 64] = A[j].x.v[k];
        fe_copy(Y[j], A[j].y);
    }
}

// Table 1P..8P of an affine P, as Jacobian points.
template <class C>
__device__ __forceinline__ void multiples8(Jac T[8], const Aff& P) {
    C::from_aff(T[0], P);
    C::dbl(T[1], T[0]);
    C::madd(T[2], T[1], P);
    C::dbl(T[3], T[1]);
    C::madd(T[4], T[3], P);
    C::dbl(T[5], T[2]);
    C::madd(T[6], T[5], P);
    C::dbl(T[7], T[3]);
}

// Compile-time loop (LLVM declines to fully unroll loops whose bodies hold several field
// multiplications, which would push the point tables out of registers into scratch).
template <int I, int N>
struct Unroll {
    template <class Fn>
    __device__ static __forceinline__ void run(Fn&& fn) {
        if constexpr (I < N) {
            fn(std::integral_constant<int, I>{});
            Unroll<I + 1, N>::run(fn);
        }
    }
};

// Rescale T[0..7] (T[0].Z == 1) to the common Z = Zc = Z1*...*Z7 without an inversion; the
// coordinates (X_j s_j^2, Y_j s_j^3), s_j = Zc / Z_j, are then AFFINE coordinates on the isomorphic
// curve E': y^2 = x^3 + b Zc^6, where a = 0 is preserved (secp256k1), so the a = 0 doubling and the
// mixed addition stay valid and the endomorphism (x, y) -> (beta x, y) still applies.  A point
// (X, Y, Z) computed on E' is (X, Y, Z * Zc) on the real curve.
__device__ __forceinline__ void coz_table_k1(Aff A[8], fe& Zc, const Jac T[8]) {
    fe pre[8], suf[8];
    FieldK1::set_one(pre[0]);
    fe_copy(pre[1], T[1].Z);
    Unroll<2, 8>::run([&](auto J) { FieldK1::mul(pre[J], pre[J - 1], T[J].Z); });   // pre[j] = Z1..Zj
    FieldK1::set_one(suf[7]);
    Unroll<0, 7>::run([&](auto J) {                                                  // suf[j] = Z(j+1)..Z7
        constexpr int j = 6 - decltype(J)::value;
        FieldK1::mul(suf[j], suf[j + 1], T[j + 1].Z);
    });
    fe_copy(Zc, pre[7]);
    Unroll<0, 8>::run([&](auto J) {
        constexpr int j = decltype(J)::value;
        fe sj, s2, s3;
        if constexpr (j == 0) fe_copy(sj, suf[0]);
        else if constexpr (j == 7) fe_copy(sj, pre[6]);
        else FieldK1::mul(sj, pre[j - 1], suf[j]);
        FieldK1::sqr(s2, sj);
        FieldK1::mul(s3, s2, sj);
        FieldK1::mul(A[j].x, T[j].X, s2);
        FieldK1::mul(A[j].y, T[j].Y, s3);
    });
}

// acc = k * P on secp256k1 via GLV: k1*P + k2*phi(P), 33 joint radix-16 Booth windows of mixed
// additions against the co-Z table; result on the real curve.
template <bool LDS = false>
__device__ __forceinline__ void glv_mul_k1(Jac& acc, const fe& k, const Aff& P, uint32_t* ldsx = nullptr) {
    fe k1, k2, Zc;
    bool neg1, neg2;
    glv_split(k1, neg1, k2, neg2, k);
    Aff A[8];
    {
        Jac T[8];
        multiples8<CurveK1>(T, P);
        coz_table_k1(A, Zc, T);
    }
    CurveK1::set_inf(acc);
    if constexpr (LDS) {
        fe Y[8];
        table_x_to_lds(ldsx, A, Y);
        add_digit_ldsx<CurveK1, FieldK1>(acc, ldsx, Y, static_cast<int>(k1.v[3] >> 31), neg1, false);
        add_digit_ldsx<CurveK1, FieldK1>(acc, ldsx, Y, static_cast<int>(k2.v[3] >> 31), neg2, true);
#pragma unroll 1
        for (int i = 31; i >= 0; --i) {
            CurveK1::dbl(acc, acc);
            CurveK1::dbl(acc, acc);
            CurveK1::dbl(acc, acc);
            CurveK1::dbl(acc, acc);
            const int d1 = booth_digit128(k1);
            const int d2 = booth_digit128(k2);
            add_digit_ldsx<CurveK1, FieldK1>(acc, ldsx, Y, d1, neg1, false);
            add_digit_ldsx<CurveK1, FieldK1>(acc, ldsx, Y, d2, neg2, true);
        }
        FieldK1::mul(acc.Z, acc.Z, Zc);
        return;
    }
    // digit 32 = bit 127 of each half
    add_digit_aff<CurveK1, FieldK1>(acc, A, static_cast<int>(k1.v[3] >> 31), neg1, false);
    add_digit_aff<CurveK1, FieldK1>(acc, A, static_cast<int>(k2.v[3] >> 31), neg2, true);
#pragma unroll 1
    for (int i = 31; i >= 0; --i) {
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        const int d1 = booth_digit128(k1);
        const int d2 = booth_digit128(k2);
        add_digit_aff<CurveK1, FieldK1>(acc, A, d1, neg1, false);
        add_digit_aff<CurveK1, FieldK1>(acc, A, d2, neg2, true);
    }
    FieldK1::mul(acc.Z, acc.Z, Zc);
}

// acc = k * P on SM2: the table 1P..8P is normalised to affine with one inversion (Montgomery's
// trick over the 7 non-trivial Z), then 65 radix-16 Booth windows of mixed additions.
// Affine table 1P..8P on SM2: multiples8 in Jacobian, then one inversion (Montgomery's trick over the
// 7 non-trivial Z).
__device__ __forceinline__ void sm2_affine_table(Aff A[8], const Aff& P) {
    Jac T[8];
    multiples8<CurveSM2>(T, P);
    fe pre[8], inv;
    FieldP2::set_one(pre[0]);
    Unroll<1, 8>::run([&](auto J) { FieldP2::mul(pre[J], pre[J - 1], T[J].Z); });
    FieldInv<FieldP2>::inv(inv, pre[7]);  // (Z1...Z7)^-1
    fe_copy(A[0].x, P.x);
    fe_copy(A[0].y, P.y);
    Unroll<0, 7>::run([&](auto J) {
        constexpr int j = 7 - decltype(J)::value;
        fe zi, zi2, zi3;
        FieldP2::mul(zi, inv, pre[j - 1]);  // Z_j^-1
        FieldP2::mul(inv, inv, T[j].Z);     // (Z1..Z(j-1))^-1
        FieldP2::sqr(zi2, zi);
        FieldP2::mul(zi3, zi2, zi);
        FieldP2::mul(A[j].x, T[j].X, zi2);
        FieldP2::mul(A[j].y, T[j].Y, zi3);
    });
}

// acc = k * P on SM2: the affine table 1P..8P, then 65 radix-16 Booth windows of mixed additions.
template <bool LDS = false>
__device__ __forceinline__ void booth_mul_sm2(Jac& acc, const fe& k_plain, const Aff& P, uint32_t* ldsx = nullptr) {
    Aff A[8];
    sm2_affine_table(A, P);
    fe k;
    fe_copy(k, k_plain);
    CurveSM2::set_inf(acc);
    if constexpr (LDS) {
        fe Y[8];
        table_x_to_lds(ldsx, A, Y);
        add_digit_ldsx<CurveSM2, FieldP2>(acc, ldsx, Y, static_cast<int>(k.v[7] >> 31), false, false);
#pragma unroll 1
        for (int i = 63; i >= 0; --i) {
            CurveSM2::dbl(acc, acc);
            CurveSM2::dbl(acc, acc);
            CurveSM2::dbl(acc, acc);
            CurveSM2::dbl(acc, acc);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, c = (top >> 27) & 1u;
            const int d = static_cast<int>(W + c) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            add_digit_ldsx<CurveSM2, FieldP2>(acc, ldsx, Y, d, false, false);
        }
        return;
    }
    add_digit_aff<CurveSM2, FieldP2>(acc, A, static_cast<int>(k.v[7] >> 31), false, false);  // digit 64
#pragma unroll 1
    for (int i = 63; i >= 0; --i) {
        CurveSM2::dbl(acc, acc);
        CurveSM2::dbl(acc, acc);
        CurveSM2::dbl(acc, acc);
        CurveSM2::dbl(acc, acc);
        const uint32_t top = k.v[7];
        const uint32_t W = top >> 28, c = (top >> 27) & 1u;
        const int d = static_cast<int>(W + c) - static_cast<int>((W >> 3) << 4);
        shl4(k);
        add_digit_aff<CurveSM2, FieldP2>(acc, A, d, false, false);
    }
}

// ------------------------------------------------------------------ table construction
template <class C, class F>
__global__ __launch_bounds__(256) void comb_table_kernel(uint32_t* tab, int sm2) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= kCombWindows * kCombEntries) return;
    const int i = idx / kCombEntries;
    uint32_t b = static_cast<uint32_t>(idx % kCombEntries);
    if (b == 0) b = 1;  // unused slot: a valid point, never selected
    fe k;
#pragma unroll
    for (int q = 0; q < 8; ++q) k.v[q] = (q == (i >> 2)) ? (b << ((i & 3) * 8)) : 0u;
    Aff G;
    fe gx, gy;
    fe_set(gx, sm2 ? kSM2Gx : kK1Gx);
    fe_set(gy, sm2 ? kSM2Gy : kK1Gy);
    fe_copy(G.x, gx);
    fe_copy(G.y, gy);
    Jac acc, S;
    C::set_inf(acc);
#pragma unroll 1
    for (int bit = 255; bit >= 0; --bit) {
        C::dbl(acc, acc);
        const bool set = (k.v[7] >> 31) != 0u;
        shl1(k);
        C::madd(S, acc, G);
        C::cmov(acc, S, set);
    }
    Aff A;
    C::to_aff(A, acc);
    F::normalize(A.x);
    F::normalize(A.y);
    uint32_t* o = tab + static_cast<size_t>(idx) * 16;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        o[w] = A.x.v[w];
        o[8 + w] = A.y.v[w];
    }
}

// 16-bit comb entry (i, b) = lo * 2^(16 i) G + hi * 2^(16 i + 8) G (b = lo + 256 hi): one addition of
// two 8-bit-table entries and one inversion.  The two addends never coincide or cancel
// (lo - 256 hi != 0 mod n), and the madd is complete anyway.
template <class C, class F>
__global__ __launch_bounds__(256) void comb_wide_kernel(uint32_t* __restrict__ wide, const uint32_t* __restrict__ tab8) {
    const uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= static_cast<uint64_t>(kWideWindows) * kWideEntries) return;
    const int i = static_cast<int>(idx / kWideEntries);
    uint32_t b = static_cast<uint32_t>(idx % kWideEntries);
    if (b == 0) b = 1;  // unused slot: a valid point, never selected
    const uint32_t lo = b & 255u, hi = b >> 8;
    Aff A, B;
    load_aff16(A, tab8 + (static_cast<size_t>(2 * i) * kCombEntries + (lo ? lo : 1u)) * 16);
    load_aff16(B, tab8 + (static_cast<size_t>(2 * i + 1) * kCombEntries + (hi ? hi : 1u)) * 16);
    Aff R;
    if (lo && hi) {
        Jac P, S;
        C::from_aff(P, A);
        C::madd(S, P, B);
        C::to_aff(R, S);
        F::normalize(R.x);
        F::normalize(R.y);
    } else {
        R = lo ? A : B;
    }
    uint32_t* o = wide + idx * 16;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        o[w] = R.x.v[w];
        o[8 + w] = R.y.v[w];
    }
}

// Kernel-selection policy, read from the environment once (at the first bcosgpu_init) and settable
// through bcosgpu_set_tx_kernel_policy (tests, tuning); never read per launch.
struct TxKernelPolicy {
    int split = -1;  // small-batch secp kernels: -1 by size (n <= 2^15), 0 never, 1 always
    int occ = 0;     // tx_verify_kernel occupancy: 0 by size (2 for n >= 2^17), 1 or 2 forced
    int coop = 1;    // small-batch secp kernel: 1 cooperative-pair, 0 4-wave split
    int f26 = 1;     // throughput secp kernels: 1 point arithmetic on the 10 x 26-bit field, 0 on FieldK1
};
static TxKernelPolicy g_policy;
static bool g_policy_read = false;

static void read_policy_env() {
    if (g_policy_read) return;
    g_policy_read = true;
    if (const char* e = getenv("BCOSGPU_TXV_SPLIT")) g_policy.split = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    if (const char* e = getenv("BCOSGPU_TXV_OCC")) g_policy.occ = (atoi(e) == 1 || atoi(e) == 2) ? atoi(e) : 0;
    if (const char* e = getenv("BCOSGPU_TXV_COOP")) g_policy.coop = atoi(e) != 0;
    if (const char* e = getenv("BCOSGPU_K1_F26")) g_policy.f26 = atoi(e) != 0;
}

void set_tx_kernel_policy(int split, int occ, int coop, int f26) {
    std::lock_guard<std::mutex> g(g_tab_mu);
    read_policy_env();
    g_policy.split = (split == 0 || split == 1) ? split : -1;
    g_policy.occ = (occ == 1 || occ == 2) ? occ : 0;
    g_policy.coop = coop != 0;
    if (f26 == 0 || f26 == 1) g_policy.f26 = f26;
}

static void free_tables(uint32_t*& a, uint32_t*& b, uint32_t*& c, uint32_t*& d) {
    for (uint32_t** p : {&a, &b, &c, &d}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
}

// init: SM2 comb table entries (x || y, R = 2^256 Montgomery domain, canonical) -> fp26's R' = 2^286
// domain: the Montgomery product (R domain) with 2^286 mod p
__device__ __constant__ static const uint32_t kSm2RtoR26[8] = {0x40000000u, 0x0u, 0xc0000000u, 0x3fffffffu,
                                                               0x0u,        0x0u, 0x0u,        0x40000000u};
__global__ __launch_bounds__(256) void sm2_table_to_r26_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                               uint64_t entries) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= entries) return;
    fe c, x, y;
    fe_set(c, kSm2RtoR26);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        x.v[w] = src[i * 16 + w];
        y.v[w] = src[i * 16 + 8 + w];
    }
    FieldP2::mul(x, x, c);
    FieldP2::mul(y, y, c);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        dst[i * 16 + w] = x.v[w];
        dst[i * 16 + 8 + w] = y.v[w];
    }
}

// Builds the device's comb tables: the 8-bit ones (512 KiB per curve) always; the 16-bit ones (64 MiB
// per curve) unless `small` or their allocation fails -- the kernels then run the 8-bit comb.
int ecc_init_tables(int device, int small) {
    std::lock_guard<std::mutex> g(g_tab_mu);
    read_policy_env();
    if (device < 0 || device >= 64) return BCOSGPU_E_ARG;
    if (g_tab_k1[device] && g_tab_sm2[device]) return 0;
    if (const char* e = getenv("BCOSGPU_TABLES")) small = small || std::strcmp(e, "small") == 0;
    uint32_t *k1 = nullptr, *sm2 = nullptr, *wk1 = nullptr, *wsm2 = nullptr;
    if (hipMalloc(&k1, kTabWords * 4) != hipSuccess || hipMalloc(&sm2, kTabWords * 4) != hipSuccess) {
        (void)hipGetLastError();
        free_tables(k1, sm2, wk1, wsm2);
        return BCOSGPU_E_HIP;
    }
    const int n = kCombWindows * kCombEntries;
    hipLaunchKernelGGL((comb_table_kernel<CurveK1, FieldK1>), dim3((n + 255) / 256), dim3(256), 0, 0, k1, 0);
    hipLaunchKernelGGL((comb_table_kernel<CurveSM2, FieldP2>), dim3((n + 255) / 256), dim3(256), 0, 0, sm2, 1);
    if (!small && (hipMalloc(&wk1, kWideTabWords * 4) != hipSuccess ||
                   hipMalloc(&wsm2, kWideTabWords * 4) != hipSuccess)) {
        (void)hipGetLastError();  // not enough memory for the wide tables: run on the 8-bit ones
        if (wk1) (void)hipFree(wk1);
        if (wsm2) (void)hipFree(wsm2);
        wk1 = wsm2 = nullptr;
    }
    if (wk1) {
        const unsigned gw = static_cast<unsigned>((static_cast<uint64_t>(kWideWindows) * kWideEntries + 255) / 256);
        hipLaunchKernelGGL((comb_wide_kernel<CurveK1, FieldK1>), dim3(gw), dim3(256), 0, 0, wk1, k1);
        hipLaunchKernelGGL((comb_wide_kernel<CurveSM2, FieldP2>), dim3(gw), dim3(256), 0, 0, wsm2, sm2);
    }
    uint32_t *sm2r = nullptr, *wsm2r = nullptr;
    if (hipMalloc(&sm2r, kTabWords * 4) != hipSuccess) {
        (void)hipGetLastError();
        free_tables(k1, sm2, wk1, wsm2);
        return BCOSGPU_E_HIP;
    }
    {
        const uint64_t ent = kTabWords / 16;
        hipLaunchKernelGGL(sm2_table_to_r26_kernel, dim3(static_cast<unsigned>((ent + 255) / 256)), dim3(256), 0, 0,
                           sm2r, sm2, ent);
    }
    if (wsm2) {
        if (hipMalloc(&wsm2r, kWideTabWords * 4) == hipSuccess) {
            const uint64_t ent = kWideTabWords / 16;
            hipLaunchKernelGGL(sm2_table_to_r26_kernel, dim3(static_cast<unsigned>((ent + 255) / 256)), dim3(256), 0,
                               0, wsm2r, wsm2, ent);
        } else {  // no room for the R'-domain copy of the wide SM2 table: every SM2 kernel on the 8-bit ones
            (void)hipGetLastError();
            wsm2r = nullptr;
        }
    }
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        free_tables(k1, sm2, wk1, wsm2);
        if (sm2r) (void)hipFree(sm2r);
        if (wsm2r) (void)hipFree(wsm2r);
        return BCOSGPU_E_HIP;
    }
    g_tab_sm2_26[device] = sm2r;
    g_wtab_sm2_26[device] = wsm2r;
    g_tab_k1[device] = k1;
    g_tab_sm2[device] = sm2;
    g_wtab_k1[device] = wk1;
    g_wtab_sm2[device] = wsm2;
    return 0;
}

// The comb tables of the current device: the 16-bit ones when present (*bits = 16), else the 8-bit
// ones (*bits = 8).
static int tables(const uint32_t** k1, const uint32_t** sm2, int* bits) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_k1[dev]) return BCOSGPU_E_NODEV;  // bcosgpu_init(dev) not called
    const bool wide = g_wtab_k1[dev] != nullptr;
    *k1 = wide ? g_wtab_k1[dev] : g_tab_k1[dev];
    *sm2 = wide ? g_wtab_sm2[dev] : g_tab_sm2[dev];
    *bits = wide ? kWideBits : 8;
    return 0;
}
// the SM2 comb table in fp26's R' domain: the 16-bit one when present, else the 8-bit one
static int tables_sm2_26(const uint32_t** tab, int* bits) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_sm2_26[dev]) return BCOSGPU_E_NODEV;
    const bool wide = g_wtab_sm2_26[dev] != nullptr;
    *tab = wide ? g_wtab_sm2_26[dev] : g_tab_sm2_26[dev];
    *bits = wide ? kWideBits : 8;
    return 0;
}
// 8-bit comb tables
static int tables8(const uint32_t** k1, const uint32_t** sm2) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_k1[dev]) return BCOSGPU_E_NODEV;
    *k1 = g_tab_k1[dev];
    *sm2 = g_tab_sm2[dev];
    return 0;
}

// ------------------------------------------------------------------ secp256k1 recover (one lane)
// libsecp256k1 secp256k1_ecdsa_recover as wedpr calls it: reject v > 3, r or s not in [1, n-1],
// (v & 2) with r >= p - n, x not on the curve, Q = infinity.  pub = (x, y) canonical, plain.
template <bool LDS = false>
__device__ __forceinline__ bool secp256k1_recover_rsv(const fe& hash_be, const fe& r, const fe& s, uint32_t v,
                                                      CombTab tab, fe& px, fe& py, uint32_t* ldsx = nullptr) {
    bool ok = v <= 3u;
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, ParamN1::M);
    fe x;
    fe_copy(x, r);
    if (v & 2u) {
        ok = ok && fe_lt_k(r, kK1PminusN);
        fe_add_k(x, r, ParamN1::M);
    }
    // y = sqrt(x^3 + 7)
    fe rhs, y, t, seven;
    FieldK1::sqr(t, x);
    FieldK1::mul(rhs, t, x);
    fe_zero(seven);
    seven.v[0] = 7;
    FieldK1::add(rhs, rhs, seven);
    FieldK1::sqrt_cand(y, rhs);
    FieldK1::sqr(t, y);
    ok = ok && FieldK1::eq(t, rhs);
    FieldK1::normalize(y);
    fe ny;
    FieldK1::neg(ny, y);
    FieldK1::normalize(ny);
    fe_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
    // u1 = -e / r, u2 = s / r (mod n)
    fe e;
    fe_copy(e, hash_be);
    reduce_once(e, ParamN1::M);
    fe rr = r;
    if (!ok) {  // keep the arithmetic well-defined on rejected lanes
        fe_zero(rr);
        rr.v[0] = 1;
    }
    fe rm, rinv, u1, u2;
    FieldN1::from_plain(rm, rr);
    FieldInv<FieldN1>::inv(rinv, rm);
    FieldN1::mul(u1, e, rinv);
    FieldN1::neg(u1, u1);
    fe ss = s;
    if (!ok) fe_zero(ss);
    FieldN1::mul(u2, ss, rinv);
    // Q = u1*G + u2*R
    Aff R;
    fe_copy(R.x, x);
    fe_copy(R.y, y);
    Jac QG, QR, Q;
    glv_mul_k1<LDS>(QR, u2, R, ldsx);
    comb_mul_rt<CurveK1>(QG, u1, tab.p, tab.bits);
    CurveK1::add(Q, QG, QR);
    ok = ok && !Q.inf;
    Aff A;
    CurveK1::to_aff(A, Q);
    FieldK1::normalize(A.x);
    FieldK1::normalize(A.y);
    fe_copy(px, A.x);
    fe_copy(py, A.y);
    return ok;
}

template <bool LDS = false>
__device__ __forceinline__ bool secp256k1_recover_lane(const fe& hash_be, const uint8_t* sig, uint32_t siglen,
                                                       CombTab tab, fe& px, fe& py, uint32_t* ldsx = nullptr) {
    if (siglen != 65u) return false;
    ByteReader rd(sig, 65);
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(i);
    fe r, s;
    fe_from_be_words(r, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(8 + i);
    fe_from_be_words(s, w);
    return secp256k1_recover_rsv<LDS>(hash_be, r, s, rd.word(16) & 0xffu, tab, px, py, ldsx);
}

}  // namespace bcosgpu
#include "recover26.h"
namespace bcosgpu {

// pub -> right160(Keccak256(pub)) as 5 little-endian memory words
__device__ __forceinline__ void keccak_address(uint32_t a[5], const fe& x, const fe& y) {
    uint32_t m[16], d[8];
    fe_to_be_words(m, x);
    fe_to_be_words(m + 8, y);
    keccak256_64(m, d);
#pragma unroll
    for (int i = 0; i < 5; ++i) a[i] = d[3 + i];
}
// pub (plain) -> right160(SM3(pub))
__device__ __forceinline__ void sm3_address(uint32_t a[5], const fe& x, const fe& y) {
    uint32_t m[16], d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        m[j] = x.v[7 - j];
        m[8 + j] = y.v[7 - j];
    }
    sm3_64(m, d);
#pragma unroll
    for (int i = 0; i < 5; ++i) a[i] = bswap32(d[3 + i]);
}

// ------------------------------------------------------------------ SM2 (one lane)
// e = SM3(Z_A || hash) as 8 big-endian words; X, Y: public key as big-endian word arrays
__device__ __forceinline__ void sm2_e(uint32_t e[8], const uint32_t X[8], const uint32_t Y[8], const fe& hash_be) {
    uint32_t V[8], W[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) V[i] = kZaMid[i];
    // block 2: bytes 128..191 = words 32..47
#pragma unroll
    for (int j = 0; j < 4; ++j) W[j] = kZaW32[j];
    W[4] = kZaC36 | (X[0] >> 16);
#pragma unroll
    for (int j = 1; j < 8; ++j) W[4 + j] = (X[j - 1] << 16) | (X[j] >> 16);
    W[12] = (X[7] << 16) | (Y[0] >> 16);
#pragma unroll
    for (int j = 1; j < 4; ++j) W[12 + j] = (Y[j - 1] << 16) | (Y[j] >> 16);
    sm3_compress(V, W);
    // block 3: words 48..63
#pragma unroll
    for (int j = 0; j < 4; ++j) W[j] = (Y[j + 3] << 16) | (Y[j + 4] >> 16);
    W[4] = (Y[7] << 16) | 0x8000u;
#pragma unroll
    for (int j = 5; j < 15; ++j) W[j] = 0;
    W[15] = 210u * 8u;
    sm3_compress(V, W);
    // e = SM3(Z_A || hash): 64 bytes -> 2 blocks
    uint32_t V2[8];
    sm3_init(V2);
#pragma unroll
    for (int j = 0; j < 8; ++j) W[j] = V[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) W[8 + j] = hash_be.v[7 - j];
    sm3_compress(V2, W);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = 0;
    W[0] = 0x80000000u;
    W[15] = 512u;
    sm3_compress(V2, W);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = V2[i];
}

// sm2_do_verify semantics (GB/T 32918.2): pub must be on the curve with coordinates < p,
// r, s in [1, n-1], t = r + s mod n != 0, accept iff (e + x1) mod n == r for (x1, y1) = sG + tP.
// The comparison is done projectively (X == (r - e mod n [+ n]) * Z^2), so no inversion.
template <bool LDS = false>
__device__ __forceinline__ bool sm2_verify_rs(const fe& hash_be, const fe& r, const fe& s, const uint32_t X[8],
                                              const uint32_t Y[8], CombTab tab, fe& px, fe& py,
                                              uint32_t* ldsx = nullptr) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        px.v[i] = X[7 - i];
        py.v[i] = Y[7 - i];
    }
    bool ok = fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    Aff P;
    FieldP2::from_plain(P.x, px);
    FieldP2::from_plain(P.y, py);
    fe b;
    fe_set(b, kSM2B);
    ok = ok && CurveSM2::on_curve(P, b);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    uint32_t eb[8];
    sm2_e(eb, X, Y, hash_be);
    fe e;
#pragma unroll
    for (int i = 0; i < 8; ++i) e.v[i] = eb[7 - i];
    reduce_once(e, ParamN2::M);
    Jac QG, QP, Q;
    booth_mul_sm2<LDS>(QP, t, P, ldsx);
    comb_mul_rt<CurveSM2>(QG, s, tab.p, tab.bits);
    CurveSM2::add(Q, QG, QP);
    ok = ok && !Q.inf;
    // x1 = X / Z^2 must be congruent to r - e (mod n): x1 = c or c + n (when c + n < p)
    fe c, c2, cm, z2, rhs;
    FieldN2::sub(c, r, e);
    FieldP2::sqr(z2, Q.Z);
    FieldP2::from_plain(cm, c);
    FieldP2::mul(rhs, cm, z2);
    bool match = FieldP2::eq(rhs, Q.X);
    const uint32_t carry = fe_add_k(c2, c, ParamN2::M);
    const bool v2 = carry == 0u && fe_lt_k(c2, ParamP2::M);
    if (v2) {
        FieldP2::from_plain(cm, c2);
        FieldP2::mul(rhs, cm, z2);
        match = match || FieldP2::eq(rhs, Q.X);
    }
    return ok && match;
}

template <bool LDS = false>
__device__ __forceinline__ bool sm2_verify_lane(const fe& hash_be, const uint8_t* sig, uint32_t siglen,
                                                CombTab tab, fe& px, fe& py, uint32_t* ldsx = nullptr) {
    if (siglen != 128u) return false;
    ByteReader rd(sig, 128);
    uint32_t w[8], X[8], Y[8];
    fe r, s;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(i);
    fe_from_be_words(r, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(8 + i);
    fe_from_be_words(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        X[i] = bswap32(rd.word(16 + i));
        Y[i] = bswap32(rd.word(24 + i));
    }
    return sm2_verify_rs<LDS>(hash_be, r, s, X, Y, tab, px, py, ldsx);
}

}  // namespace bcosgpu
#include "verify_sm2_26.h"
namespace bcosgpu {

// ------------------------------------------------------------------ secp256k1 verify (known key)
// libsecp256k1 secp256k1_ecdsa_verify as wedpr_secp256k1_verify calls it (Secp256k1Crypto.cpp:51-63):
// pub (x, y) < p on the curve, r, s in [1, n-1], low-S (s <= n/2), e = hash mod n,
// (x1, .) = (e/s) G + (r/s) P, accept iff x1 mod n == r.  Only bytes 0..63 of the signature (r || s)
// are read.  The comparison is projective (X == r Z^2, or (r + n) Z^2 when r + n < p): no inversion.
__device__ __constant__ static const uint32_t kN1HalfPlus[8] = {0x681b20a1u, 0xdfe92f46u, 0x57a4501du, 0x5d576e73u,
                                                            0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
__device__ __forceinline__ bool secp256k1_verify_lane(const fe& hash_be, const uint8_t* sig, const uint8_t* pub,
                                                      CombTab tab) {
    ByteReader rs(sig, 64), rp(pub, 64);
    uint32_t w[8];
    fe r, s, x, y;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rs.word(i);
    fe_from_be_words(r, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rs.word(8 + i);
    fe_from_be_words(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rp.word(i);
    fe_from_be_words(x, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rp.word(8 + i);
    fe_from_be_words(y, w);
    bool ok = fe_lt_k(x, FieldK1::P) && fe_lt_k(y, FieldK1::P);
    {
        fe l, rr, t, seven;
        FieldK1::sqr(l, y);
        FieldK1::sqr(t, x);
        FieldK1::mul(rr, t, x);
        fe_zero(seven);
        seven.v[0] = 7;
        FieldK1::add(rr, rr, seven);
        ok = ok && FieldK1::eq(l, rr);
    }
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, kN1HalfPlus);
    fe e;
    fe_copy(e, hash_be);
    reduce_once(e, ParamN1::M);
    fe ss = s;
    if (!ok) {  // keep the arithmetic well-defined on rejected lanes
        fe_zero(ss);
        ss.v[0] = 1;
    }
    fe sm, sinv, u1, u2;
    FieldN1::from_plain(sm, ss);
    FieldInv<FieldN1>::inv(sinv, sm);
    FieldN1::mul(u1, e, sinv);
    FieldN1::mul(u2, r, sinv);
    Aff P;
    fe_copy(P.x, x);
    fe_copy(P.y, y);
    if (!ok) {  // a valid point for the rejected lanes
        fe_set(P.x, kK1Gx);
        fe_set(P.y, kK1Gy);
    }
    Jac QG, QP, Q;
    glv_mul_k1(QP, u2, P);
    comb_mul_rt<CurveK1>(QG, u1, tab.p, tab.bits);
    CurveK1::add(Q, QG, QP);
    ok = ok && !Q.inf;
    fe z2, rhs, r2;
    FieldK1::sqr(z2, Q.Z);
    FieldK1::mul(rhs, r, z2);
    bool match = FieldK1::eq(rhs, Q.X);
    const uint32_t carry = fe_add_k(r2, r, ParamN1::M);
    if (carry == 0u && fe_lt_k(r2, FieldK1::P)) {
        FieldK1::mul(rhs, r2, z2);
        match = match || FieldK1::eq(rhs, Q.X);
    }
    return ok && match;
}

// secp256k1_verify_lane with the point arithmetic on fe26 (same decisions and result)
__device__ __forceinline__ bool secp256k1_verify_lane26(const fe& hash_be, const uint8_t* sig, const uint8_t* pub,
                                                        CombTab tab) {
    ByteReader rs(sig, 64), rp(pub, 64);
    uint32_t w[8];
    fe r, s, x, y;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rs.word(i);
    fe_from_be_words(r, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rs.word(8 + i);
    fe_from_be_words(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rp.word(i);
    fe_from_be_words(x, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rp.word(8 + i);
    fe_from_be_words(y, w);
    bool ok = fe_lt_k(x, FieldK1::P) && fe_lt_k(y, FieldK1::P);
    Aff26 P;
    fe26_from_fe(P.x, x);
    fe26_from_fe(P.y, y);
    {
        fe26 l, rr, t, seven;
        fe26_sqr(l, P.y);
        fe26_sqr(t, P.x);
        fe26_mul(rr, t, P.x);
        fe26_set_small(seven, 7u);
        fe26_add(rr, rr, seven);
        fe26_sub<3>(l, l, rr);
        ok = ok && fe26_is_zero(l);
    }
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, kN1HalfPlus);
    fe e;
    fe_copy(e, hash_be);
    reduce_once(e, ParamN1::M);
    fe ss = s;
    if (!ok) {
        fe_zero(ss);
        ss.v[0] = 1;
    }
    fe sm, sinv, u1, u2;
    FieldN1::from_plain(sm, ss);
    FieldInv<FieldN1>::inv(sinv, sm);
    FieldN1::mul(u1, e, sinv);
    FieldN1::mul(u2, r, sinv);
    if (!ok) {
        fe26_const(P.x, kK1Gx);
        fe26_const(P.y, kK1Gy);
    }
    Jac26 QG, QP, Q;
    glv_mul_k1_26<false>(QP, u2, P, nullptr);
    comb_mul26_rt(QG, u1, tab);
    CurveK1x::add(Q, QG, QP);  // X m 6
    ok = ok && !Q.inf;
    fe26 z2, rhs, R, d;
    fe26_sqr(z2, Q.Z);
    fe26_from_fe(R, r);
    fe26_mul(rhs, R, z2);
    fe26_sub<7>(d, rhs, Q.X);
    bool match = fe26_is_zero(d);
    fe r2;
    const uint32_t carry = fe_add_k(r2, r, ParamN1::M);
    if (carry == 0u && fe_lt_k(r2, FieldK1::P)) {
        fe26_from_fe(R, r2);
        fe26_mul(rhs, R, z2);
        fe26_sub<7>(d, rhs, Q.X);
        match = match || fe26_is_zero(d);
    }
    return ok && match;
}

// ------------------------------------------------------------------ kernels
template <bool F26>
__global__ __launch_bounds__(256) void secp256k1_recover_kernel(const uint8_t* __restrict__ hash,
                                                                const uint8_t* __restrict__ sig, uint32_t stride,
                                                                uint64_t n, const uint32_t* __restrict__ tab, int tbits,
                                                                uint8_t* __restrict__ pub, uint8_t* __restrict__ addr,
                                                                uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe h, x, y;
    load_be256_aligned(h, hash + 32 * i);
    const bool ok = F26 ? secp256k1_recover_lane26(h, sig + static_cast<uint64_t>(stride) * i, 65u, CombTab{tab, tbits}, x, y)
                        : secp256k1_recover_lane(h, sig + static_cast<uint64_t>(stride) * i, 65u, CombTab{tab, tbits}, x, y);
    if (!ok) {
        fe_zero(x);
        fe_zero(y);
    }
    if (pub) {
        store_be256(pub + 64 * i, x);
        store_be256(pub + 64 * i + 32, y);
    }
    if (addr) {
        uint32_t a[5] = {0, 0, 0, 0, 0};
        if (ok) keccak_address(a, x, y);
        uint32_t* o = reinterpret_cast<uint32_t*>(addr + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = a[k];
    }
    okout[i] = ok ? 1 : 0;
}

template <bool F26>
__global__ __launch_bounds__(256) void sm2_verify_kernel(const uint8_t* __restrict__ hash,
                                                         const uint8_t* __restrict__ sig, uint32_t stride,
                                                         uint64_t n, const uint32_t* __restrict__ tab, int tbits,
                                                         uint8_t* __restrict__ addr, uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe h, x, y;
    load_be256_aligned(h, hash + 32 * i);
    const bool ok = F26 ? sm2_verify_lane26(h, sig + static_cast<uint64_t>(stride) * i, 128u, CombTab{tab, tbits}, x, y)
                        : sm2_verify_lane(h, sig + static_cast<uint64_t>(stride) * i, 128u, CombTab{tab, tbits}, x, y);
    if (addr) {
        uint32_t a[5] = {0, 0, 0, 0, 0};
        if (ok) sm3_address(a, x, y);
        uint32_t* o = reinterpret_cast<uint32_t*>(addr + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = a[k];
    }
    okout[i] = ok ? 1 : 0;
}

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

// EVM ecRecover precompile (bcos-executor/src/vm/Precompiled.cpp:443-482) for a batch: input =
// hash(32) || v(32) || r(32) || s(32); recid = (byte)(in[63] - 27) (the other 31 bytes of v are not
// read); on success out = 12 zero bytes || right160(Keccak256(pub)), ok = 1; on failure the
// precompile returns an empty output: out = zeros, ok = 0.
template <bool F26>
__global__ __launch_bounds__(256) void ecrecover_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                        const uint32_t* __restrict__ tab, int tbits,
                                                        uint8_t* __restrict__ out, uint8_t* __restrict__ okout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = in + 128 * i;
    fe h, r, s, x, y;
    load_be256_aligned(h, p);
    load_be256_aligned(r, p + 64);
    load_be256_aligned(s, p + 96);
    const uint32_t v = (reinterpret_cast<const uint32_t*>(p)[15] >> 24) - 27u;
    const bool ok = F26 ? secp256k1_recover_rsv26(h, r, s, v & 0xffu, CombTab{tab, tbits}, x, y)
                        : secp256k1_recover_rsv(h, r, s, v & 0xffu, CombTab{tab, tbits}, x, y);
    uint32_t a[5] = {0, 0, 0, 0, 0};
    if (ok) keccak_address(a, x, y);
    uint32_t* o = reinterpret_cast<uint32_t*>(out + 32 * i);
#pragma unroll
    for (int k = 0; k < 3; ++k) o[k] = 0u;
#pragma unroll
    for (int k = 0; k < 5; ++k) o[3 + k] = a[k];
    okout[i] = ok ? 1 : 0;
}

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

// ------------------------------------------------------------------ split (latency) secp256k1 tx verify
// Small batches are latency-bound: 10k txs fill 157 waves on 1,024 SIMDs, so one recovery per lane
// leaves most of the chip idle.  Here a 256-thread workgroup owns 64 txs and its 4 waves (on the
// CU's 4 SIMDs) run independent parts of every recovery concurrently, exchanging through LDS:
//   phase A  wave 1: tx hash, r^-1 (safegcd), u1 = -e/r, u2 = s/r, GLV split of u2
//            wave 2: y = sqrt(x^3 + 7), table 1R..8R, co-Z rescale -> LDS (affine on E')
//   phase C  wave 0: k1 * R      wave 1: k2 * phi(R)   (32 radix-16 windows each, table in LDS)
//            wave 2: u1 * G (comb)
//   phase D  wave 0: sum on E', map to E, add the G part, affine, Keccak address, store
// Results are bit-identical to tx_verify_kernel<0, *>.
struct SplitLds {
    uint32_t tab[8][16][64];  // [entry][x0..7, y0..7][lane]: conflict-free per-lane gathers
    uint32_t zc[8][64];
    uint32_t u1[8][64];
    uint32_t k1[4][64];
    uint32_t k2[4][64];
    uint32_t flags[64];       // bit0 wave-1 checks ok, bit1 wave-2 checks ok, bit2 neg1, bit3 neg2
    uint32_t pt[3][25][64];   // partial results: X, Y, Z, inf
};

__device__ __forceinline__ void lds_store_fe(uint32_t (*dst)[64], const fe& a, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k][lane] = a.v[k];
}
__device__ __forceinline__ void lds_load_fe(fe& a, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a.v[k] = src[k][lane];
}
__device__ __forceinline__ void lds_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
    lds_store_fe(dst, P.X, lane);
    lds_store_fe(dst + 8, P.Y, lane);
    lds_store_fe(dst + 16, P.Z, lane);
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void lds_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
    lds_load_fe(P.X, src, lane);
    lds_load_fe(P.Y, src + 8, lane);
    lds_load_fe(P.Z, src + 16, lane);
    P.inf = src[24][lane] != 0u;
}

// acc += (+-d) (phi ? lambda : 1) T[|d| - 1], T gathered per lane from the LDS table (on E')
__device__ __forceinline__ void add_digit_lds(Jac& acc, const SplitLds& L, int lane, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (16 * 64) + lane;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = base[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    if (phi) {
        fe b;
        fe_set(b, kGlvBeta);
        FieldK1::mul(S.x, S.x, b);
    }
    fe ny;
    FieldK1::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    CurveK1::madd(R, acc, S);
    CurveK1::cmov(acc, R, d != 0);
}

__device__ __forceinline__ void glv_half_lds(Jac& acc, fe& k, bool neg, bool phi, const SplitLds& L, int lane) {
    CurveK1::set_inf(acc);
    add_digit_lds(acc, L, lane, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
    for (int i = 31; i >= 0; --i) {
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        add_digit_lds(acc, L, lane, booth_digit128(k), neg, phi);
    }
}

// parse r, s, v of a 65-byte signature; ok = libsecp256k1 parse_compact + r, s != 0
__device__ __forceinline__ bool parse_sig65(const uint8_t* sig, uint32_t siglen, fe& r, fe& s, uint32_t& v) {
    if (siglen != 65u) {
        fe_zero(r);
        fe_zero(s);
        v = 0;
        return false;
    }
    ByteReader rd(sig, 65);
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(i);
    fe_from_be_words(r, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = rd.word(8 + i);
    fe_from_be_words(s, w);
    v = rd.word(16) & 0xffu;
    return v <= 3u && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, ParamN1::M);
}

__global__ __launch_bounds__(256, 1) void tx_verify_split_kernel(const uint8_t* __restrict__ pre,
                                                                 const uint64_t* __restrict__ pre_off,
                                                                 const uint8_t* __restrict__ sig,
                                                                 const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                 const uint32_t* __restrict__ tab,
                                                                 uint8_t* __restrict__ txhash,
                                                                 uint8_t* __restrict__ sender,
                                                                 uint8_t* __restrict__ status) {
    __shared__ SplitLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    uint64_t sa = 0, sb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
    }
    const uint32_t slen = (sb - sa) > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(sb - sa);
    // ---------------------------------------------------------------- phase A
    if (wave == 1) {
        if (active) {
            const uint64_t a = pre_off[i], b = pre_off[i + 1];
            const uint32_t len = static_cast<uint32_t>(b - a);
            ByteReader rd(pre + a, len);
            uint32_t d[8];
            keccak256_msg(rd, len, d);
            store_digest(KECCAK256, txhash + 32 * i, d);
            fe e, r, s;
            uint32_t v;
            fe_from_be_words(e, d);
            reduce_once(e, ParamN1::M);
            const bool ok = parse_sig65(sig + sa, slen, r, s, v);
            if (!ok) {
                fe_zero(r);
                r.v[0] = 1;
                fe_zero(s);
            }
            fe rm, rinv, u1, u2, k1, k2;
            FieldN1::from_plain(rm, r);
            FieldInv<FieldN1>::inv(rinv, rm);
            FieldN1::mul(u1, e, rinv);
            FieldN1::neg(u1, u1);
            FieldN1::mul(u2, s, rinv);
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
            lds_store_fe(L.u1, u1, lane);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                L.k1[k][lane] = k1.v[k];
                L.k2[k][lane] = k2.v[k];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
    } else if (wave == 2) {
        if (active) {
            fe r, s;
            uint32_t v;
            bool ok = parse_sig65(sig + sa, slen, r, s, v);
            fe x;
            fe_copy(x, r);
            if (v & 2u) {
                ok = ok && fe_lt_k(r, kK1PminusN);
                fe_add_k(x, r, ParamN1::M);
            }
            fe rhs, y, t, seven;
            FieldK1::sqr(t, x);
            FieldK1::mul(rhs, t, x);
            fe_zero(seven);
            seven.v[0] = 7;
            FieldK1::add(rhs, rhs, seven);
            FieldK1::sqrt_cand(y, rhs);
            FieldK1::sqr(t, y);
            ok = ok && FieldK1::eq(t, rhs);
            FieldK1::normalize(y);
            fe ny;
            FieldK1::neg(ny, y);
            FieldK1::normalize(ny);
            fe_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            Aff R, A[8];
            fe_copy(R.x, x);
            fe_copy(R.y, y);
            fe Zc;
            {
                Jac T[8];
                multiples8<CurveK1>(T, R);
                coz_table_k1(A, Zc, T);
            }
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
            });
            lds_store_fe(L.zc, Zc, lane);
            L.pt[2][24][lane] = ok ? 2u : 0u;  // wave-2 verdict travels in a scratch slot until phase C
        }
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase C
    uint32_t flags = 0;
    if (active) flags = L.flags[lane] | L.pt[2][24][lane];
    __syncthreads();
    if (wave <= 1) {
        if (active) {
            fe k;
            fe_zero(k);
#pragma unroll
            for (int q = 0; q < 4; ++q) k.v[q] = wave == 0 ? L.k1[q][lane] : L.k2[q][lane];
            const bool neg = wave == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
            Jac P;
            glv_half_lds(P, k, neg, wave == 1, L, lane);
            lds_store_jac(L.pt[wave], P, lane);
        }
    } else if (wave == 2) {
        if (active) {
            fe u1;
            lds_load_fe(u1, L.u1, lane);
            Jac PG;
            comb_mul<CurveK1, 8>(PG, u1, tab);
            lds_store_jac(L.pt[2], PG, lane);
        }
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase D
    if (wave == 0 && active) {
        Jac P0, P1, PG, Q, R;
        lds_load_jac(P0, L.pt[0], lane);
        lds_load_jac(P1, L.pt[1], lane);
        lds_load_jac(PG, L.pt[2], lane);
        fe Zc;
        lds_load_fe(Zc, L.zc, lane);
        CurveK1::add(Q, P0, P1);  // on E'
        FieldK1::mul(Q.Z, Q.Z, Zc);  // -> E
        CurveK1::add(R, Q, PG);
        const bool ok = (flags & 3u) == 3u && !R.inf;
        Aff A;
        CurveK1::to_aff(A, R);
        FieldK1::normalize(A.x);
        FieldK1::normalize(A.y);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok) keccak_address(ad, A.x, A.y);
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ad[k];
        status[i] = ok ? 0 : 1;
    }
}

// ------------------------------------------------------------------ cooperative (latency) secp256k1 tx verify
// A lone wave on a SIMD issues a Comba step only every ~15 cycles and a 64-bit-result op every ~10
// (profiles/r01_mulbench.json), so C2's one-wave-per-SIMD batches are bound by the length of the
// serial point-operation chain, not by the SIMD.  Here the two GLV halves each run on a PAIR of
// waves that split every doubling and mixed addition by dependency level and trade intermediate
// field elements through LDS:
//   dbl  (3M + 4S, depth 2): a: A = X^2, F = (3A)^2, Z3 = 2 Y Z | b: B = Y^2, D = 4 X B, 8 B^2
//                            -> both: X3, Y3 = E (D - X3) - 8C        4 instead of 7, one barrier
//   madd (7M + 4S):          a: Z1Z1, U2, HH, Z3 | b: Z1Z1, S2', S2, rr^2 -> a: J | b: V
//                            -> a: rr (V - X3) | b: Y J        6 instead of 11
// Both waves of a pair hold the whole point after every operation (they compute bit-identical
// values), so the four waves run the same barrier schedule.  Phase A needs no square root before
// the table (the R chain runs on an isomorphic curve, see phase A), so the hash, r^-1, the R table,
// the square root and the comb windows of u1*G run side by side on the four waves, and phase C is
// the two cooperative GLV chains only.  Bit-identical to tx_verify_kernel<0, *>.
#ifdef BCOSGPU_COOP_TIMING  // tools/coopbench.hip: phase timestamps of workgroup 0
__device__ uint64_t g_coop_t[4][8];
__device__ uint64_t g_dbl_t[4][8];
#define DBL_T(k) \
    if (c.probe && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][k] = clock64()
#define COOP_T(k) \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_coop_t[threadIdx.x >> 6][k] = clock64()
#else
#define COOP_T(k) \
    do {          \
    } while (0)
#define DBL_T(k) \
    do {         \
    } while (0)
#endif
struct CoopLds {
    uint32_t tab[8][16][64];          // co-Z table on E': [entry][x0..7, y0..7][lane]
    uint32_t zc[8][64];
    uint32_t k[2][4][64];             // GLV halves
    uint32_t flags[64];               // bit0 scalars ok, bit1 R ok, bit2 neg1, bit3 neg2
    uint4 ex[2][2][6][2][64];         // [chain][writer role][slot][word quad][lane]; madd: 0-2 exchange 0, 3: 1, 4: 2; dbl: 0-2 | 3-5
    uint32_t tabphx[8][8][64];        // beta * x of the table entries (chain 1's phi(R) table)
    uint32_t pt[5][25][64];           // chain results 0/1, G partials 2..4 (X, Y, Z, inf)
    uint32_t xe[8][64];               // e = H(m) mod n (wave 3 -> waves 0, 1)
    uint32_t xrinv[8][64];            // r^-1, Montgomery form (wave 0 -> waves 1, 3)
    uint32_t ys[8][64];               // y of R with v's parity (wave 2 -> phase D)
    uint32_t rflag[64];               // R verdict (wave 2)
    uint32_t post[2];                 // phase-A hand-off flags: 0 r^-1 ready, 1 e ready
};

// One-way hand-offs between waves inside phase A: the producer writes its per-lane values, then
// releases the flag; the consumer acquires it.  Workgroup scope, so these are LDS-only fences.
__device__ __forceinline__ void coop_post(uint32_t* f) {
    __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void coop_wait(uint32_t* f) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(1);
}

struct CoopCtx {
    CoopLds* L;
    int chain, role, lane;
    bool probe;  // BCOSGPU_COOP_TIMING: stamp the doubling phases (workgroup 0, one doubling)
    // An exchange slot is rewritten only after the barrier that follows the partner's read of it,
    // so one slot per (exchange, field element) suffices across consecutive operations.
    // Layout [quad][lane] of uint4: one fe is two conflict-free ds_write_b128 / ds_read_b128.
    __device__ __forceinline__ uint4* slot(int x, int r, int f) const {
        return &L->ex[chain][r][x == 0 ? f : 2 + x][0][0] + lane;
    }
    __device__ __forceinline__ void put(int x, int f, const fe& a) const {
        uint4* p = slot(x, role, f);
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void puts(int s, const fe& a) const {  // raw slot index 0..5
        uint4* p = &L->ex[chain][role][s][0][0] + lane;
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void gets(int s, fe& a) const {
        const uint4* p = &L->ex[chain][role ^ 1][s][0][0] + lane;
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
    __device__ __forceinline__ void get(int x, int f, fe& a) const {  // the partner's value
        const uint4* p = slot(x, role ^ 1, f);
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
};

// P = 2 P (a = 0, dbl-2009-l with D = 4 X B), P replicated on both waves of the pair; ONE exchange:
//   a: A = X^2, E = 3A, F = E^2, Z3 = 2 Y Z | b: B = Y^2, D = 4 X B, C = B^2, C8 = 8 C
//   -> both: X3 = F - 2D, Y3 = E (D - X3) - C8
// The shifted passes (shl<k>, mul3) replace ten field additions.  S0 is the exchange buffer: slots
// 0-2 (shared with coop_madd's exchange 0) or 3-5 (3, 4 shared with its exchanges 1, 2).  The four
// doublings of a window use 0, 3, 0, 3, so a slot is rewritten only after the barrier that follows
// the partner's last read of it (the madd rewrites 0-2 before its first barrier, two doublings after
// the last read of buffer 0, and 3/4 only after its first/second barrier).
template <int S0>
__device__ __forceinline__ void coop_dbl(Jac& P, const CoopCtx& c) {
    fe E, F, D, C8, Z3, X3, Y3, t;
    DBL_T(0);
    if (c.role == 0) {
        fe A;
        FieldK1::sqr(A, P.X);
        FieldK1::mul3(E, A);
        FieldK1::sqr(F, E);
        c.puts(S0, E);
        c.puts(S0 + 1, F);
        FieldK1::mul(Z3, P.Y, P.Z);
        FieldK1::template shl<1>(Z3, Z3);
        c.puts(S0 + 2, Z3);
    } else {
        fe B, C;
        FieldK1::sqr(B, P.Y);
        FieldK1::mul(D, P.X, B);
        FieldK1::template shl<2>(D, D);
        c.puts(S0, D);
        FieldK1::sqr(C, B);
        FieldK1::template shl<3>(C8, C);
        c.puts(S0 + 1, C8);
    }
    DBL_T(1);
    __syncthreads();
    DBL_T(2);
    if (c.role == 0) {
        c.gets(S0, D);
        c.gets(S0 + 1, C8);
    } else {
        c.gets(S0, E);
        c.gets(S0 + 1, F);
        c.gets(S0 + 2, Z3);
    }
    FieldK1::template shl<1>(t, D);
    FieldK1::sub(X3, F, t);
    FieldK1::sub(t, D, X3);
    FieldK1::mul(Y3, E, t);
    FieldK1::sub(Y3, Y3, C8);
    DBL_T(3);
    fe_copy(P.X, X3);
    fe_copy(P.Y, Y3);
    fe_copy(P.Z, Z3);
    DBL_T(4);
}

// P = P + Q (madd-2007-bl with the complete-addition special cases of CurveK1::madd), Q affine.
__device__ __forceinline__ void coop_madd(Jac& R, const Jac& P, const Aff& Q, const CoopCtx& c) {
    fe Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    FieldK1::sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        FieldK1::mul(u, Q.x, Z1Z1);       // U2
        FieldK1::sub(H, u, P.X);
        FieldK1::sqr(HH, H);
        FieldK1::add(t, P.Z, H);
        FieldK1::sqr(Z3, t);
        FieldK1::sub(Z3, Z3, Z1Z1);
        FieldK1::sub(Z3, Z3, HH);
        c.put(0, 0, H);
        c.put(0, 1, HH);
        c.put(0, 2, Z3);
    } else {
        FieldK1::mul(u, Q.y, P.Z);
        FieldK1::mul(u, u, Z1Z1);         // S2
        FieldK1::sub(rr, u, P.Y);
        FieldK1::template shl<1>(rr, rr);
        FieldK1::sqr(R2, rr);
        c.put(0, 0, rr);
        c.put(0, 1, R2);
    }
    __syncthreads();
    if (c.role == 0) {
        c.get(0, 0, rr);
        c.get(0, 1, R2);
    } else {
        c.get(0, 0, H);
        c.get(0, 1, HH);
        c.get(0, 2, Z3);
    }
    FieldK1::template shl<2>(I, HH);
    if (c.role == 0) {
        FieldK1::mul(J, H, I);
        c.put(1, 0, J);
    } else {
        FieldK1::mul(V, P.X, I);
        c.put(1, 0, V);
    }
    __syncthreads();
    if (c.role == 0) c.get(1, 0, V);
    else c.get(1, 0, J);
    FieldK1::sub(X3, R2, J);
    FieldK1::template shl<1>(t, V);
    FieldK1::sub(X3, X3, t);
    if (c.role == 0) {
        FieldK1::sub(t, V, X3);
        FieldK1::mul(u, rr, t);           // rr (V - X3)
        c.put(2, 0, u);
    } else {
        FieldK1::mul(u, P.Y, J);
        FieldK1::template shl<1>(u, u);   // 2 Y J
        c.put(2, 0, u);
    }
    __syncthreads();
    if (c.role == 0) {
        c.get(2, 0, t);
        FieldK1::sub(Y3, u, t);
    } else {
        c.get(2, 0, t);
        FieldK1::sub(Y3, t, u);
    }
    // special cases, as CurveK1::madd (computed identically on both waves, no barriers)
    const bool hz = FieldK1::is_zero(H) && !P.inf;
    const bool rz = FieldK1::is_zero(rr);
    Jac D;
    if (hz && rz) CurveK1::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe_copy(R.X, X3);
    fe_copy(R.Y, Y3);
    fe_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveK1::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe_copy(R.X, Q.x);
        fe_copy(R.Y, Q.y);
        FieldK1::set_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void coop_add_digit(Jac& acc, const CoopCtx& c, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    const uint32_t* bx = phi ? &c.L->tabphx[0][0][0] + m * (8 * 64) + c.lane : base;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = bx[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    fe ny;
    FieldK1::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    coop_madd(R, acc, S, c);
    CurveK1::cmov(acc, R, d != 0);
}

// acc = u1 * G restricted to comb windows [lo, hi)
__device__ __forceinline__ void comb_range_k1(Jac& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo, int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    CurveK1::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        const uint4* e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        const uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
        Aff T;
        T.x.v[0] = q0.x; T.x.v[1] = q0.y; T.x.v[2] = q0.z; T.x.v[3] = q0.w;
        T.x.v[4] = q1.x; T.x.v[5] = q1.y; T.x.v[6] = q1.z; T.x.v[7] = q1.w;
        T.y.v[0] = q2.x; T.y.v[1] = q2.y; T.y.v[2] = q2.z; T.y.v[3] = q2.w;
        T.y.v[4] = q3.x; T.y.v[5] = q3.y; T.y.v[6] = q3.z; T.y.v[7] = q3.w;
        Jac S;
        CurveK1::madd(S, acc, T);
        CurveK1::cmov(acc, S, b != 0u);
    }
}

__device__ __forceinline__ void coop_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = P.X.v[k];
        dst[8 + k][lane] = P.Y.v[k];
        dst[16 + k][lane] = P.Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void coop_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        P.X.v[k] = src[k][lane];
        P.Y.v[k] = src[8 + k][lane];
        P.Z.v[k] = src[16 + k][lane];
    }
    P.inf = src[24][lane] != 0u;
}

__global__ __launch_bounds__(256, 1) void tx_verify_coop_kernel(const uint8_t* __restrict__ pre,
                                                                const uint64_t* __restrict__ pre_off,
                                                                const uint8_t* __restrict__ sig,
                                                                const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                const uint32_t* __restrict__ tab,
                                                                uint8_t* __restrict__ txhash,
                                                                uint8_t* __restrict__ sender,
                                                                uint8_t* __restrict__ status) {
    __shared__ CoopLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    COOP_T(0);
    uint64_t sa = 0, sb = 0, pa = 0, pb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
        pa = pre_off[i];
        pb = pre_off[i + 1];
    }
    const uint32_t slen = (sb - sa) > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(sb - sa);
    if (threadIdx.x == 0) {
        L.post[0] = 0u;
        L.post[1] = 0u;
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase A
    // R = (x, y) is needed through y only at the very end: the R chain runs on the isomorphic curve
    // E_w: Y^2 = X^3 + 7 w^3 (w = x^3 + 7), where R' = (w x, w^2) needs no square root, and a point
    // (X, Y, Z) of E_w is (X, Y, Z y) on E.  So the square root runs beside the table instead of
    // before it.  Schedule: wave 0 inverts r, wave 3 hashes (they swap r^-1 and e through LDS flags),
    // wave 1 builds the R' table and then the GLV split, wave 2 takes the square root; the comb
    // windows of u1 * G go to waves 0 and 3 and the tail of wave 1.
    fe r, s;
    uint32_t v = 0;
    bool ok = false;
    if (active) ok = parse_sig65(sig + sa, slen, r, s, v);
    else { fe_zero(r); fe_zero(s); }
    if (wave == 1 || wave == 2) {
        fe x, rhs, t, seven;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        FieldK1::sqr(t, x);
        FieldK1::mul(rhs, t, x);
        fe_zero(seven);
        seven.v[0] = 7;
        FieldK1::add(rhs, rhs, seven);  // w
        if (wave == 2) {
            fe y;
            FieldK1::sqrt_cand(y, rhs);
            FieldK1::sqr(t, y);
            okr = okr && FieldK1::eq(t, rhs);
            FieldK1::normalize(y);
            fe ny;
            FieldK1::neg(ny, y);
            FieldK1::normalize(ny);
            fe_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            lds_store_fe(L.ys, y, lane);
            L.rflag[lane] = okr ? 2u : 0u;
            COOP_T(6);
        } else {
            Aff R, A[8];
            FieldK1::mul(R.x, rhs, x);  // w x
            FieldK1::sqr(R.y, rhs);     // w^2
            fe Zc;
            {
                Jac T[8];
                multiples8<CurveK1>(T, R);
                coz_table_k1(A, Zc, T);
            }
            fe beta;
            fe_set(beta, kGlvBeta);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
                fe bx;
                FieldK1::mul(bx, A[j].x, beta);
                lds_store_fe(L.tabphx[j], bx, lane);
            });
            lds_store_fe(L.zc, Zc, lane);
            COOP_T(6);
        }
    }
    if (!ok) {  // scalars of a rejected signature: any well-defined values (the verdict is already 1)
        fe_zero(r);
        r.v[0] = 1;
        fe_zero(s);
    }
    if (wave == 3) {
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            keccak256_msg(rd, len, d);
            store_digest(KECCAK256, txhash + 32 * i, d);
        }
        fe e;
        fe_from_be_words(e, d);
        reduce_once(e, ParamN1::M);
        lds_store_fe(L.xe, e, lane);
        coop_post(&L.post[1]);
        COOP_T(7);
    } else if (wave == 0) {
        fe rm, rinv;
        FieldN1::from_plain(rm, r);
        FieldInv<FieldN1>::inv(rinv, rm);
        lds_store_fe(L.xrinv, rinv, lane);
        coop_post(&L.post[0]);
        COOP_T(7);
    }
    if (wave != 2) {
        coop_wait(&L.post[0]);
        coop_wait(&L.post[1]);
        fe e, rinv, u1;
        lds_load_fe(e, L.xe, lane);
        lds_load_fe(rinv, L.xrinv, lane);
        FieldN1::mul(u1, e, rinv);
        FieldN1::neg(u1, u1);
        if (wave == 1) {
            fe u2, k1, k2;
            FieldN1::mul(u2, s, rinv);
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L.k[0][q][lane] = k1.v[q];
                L.k[1][q][lane] = k2.v[q];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
        // comb windows of u1 * G: wave 0 [0, kCombW0), wave 3 [kCombW0, kCombW1), wave 1 [kCombW1, 32)
        constexpr int kCombW0 = 12, kCombW1 = 24;
        Jac G;
        const int lo = wave == 0 ? 0 : wave == 3 ? kCombW0 : kCombW1;
        const int hi = wave == 0 ? kCombW0 : wave == 3 ? kCombW1 : 32;
        comb_range_k1(G, u1, tab, lo, hi);
        coop_store_jac(L.pt[wave == 0 ? 2 : wave == 3 ? 3 : 4], G, lane);
    }
    COOP_T(1);
    __syncthreads();
    // ---------------------------------------------------------------- phase C: two cooperative GLV chains
    const uint32_t flags = L.flags[lane] | L.rflag[lane];
    CoopCtx c{&L, wave >> 1, wave & 1, lane, false};
    fe k;
    fe_zero(k);
#pragma unroll
    for (int q = 0; q < 4; ++q) k.v[q] = L.k[c.chain][q][lane];
    const bool neg = c.chain == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
    const bool phi = c.chain == 1;
    Jac acc;
    CurveK1::set_inf(acc);
    coop_add_digit(acc, c, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
    for (int w = 31; w >= 0; --w) {
        coop_dbl<0>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = blockIdx.x == 0 && w == 20;
#endif
        coop_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = false;
#endif
        coop_dbl<0>(acc, c);
        coop_dbl<3>(acc, c);
        coop_add_digit(acc, c, booth_digit128(k), neg, phi);
    }
    COOP_T(2);
    if (c.role == 0) coop_store_jac(L.pt[c.chain], acc, lane);
    __syncthreads();
    // ---------------------------------------------------------------- phase D
    if (wave == 1) {  // G part: partials 0 + 1 + 2
        Jac G0, G1, T, U;
        coop_load_jac(G0, L.pt[2], lane);
        coop_load_jac(G1, L.pt[3], lane);
        CurveK1::add(T, G0, G1);
        coop_load_jac(G0, L.pt[4], lane);
        CurveK1::add(U, T, G0);
        coop_store_jac(L.pt[2], U, lane);
    } else if (wave == 0) {  // R part: co-Z curve -> E_w (Z * Zc) -> E (Z * y)
        Jac P0, P1, Q;
        coop_load_jac(P0, L.pt[0], lane);
        coop_load_jac(P1, L.pt[1], lane);
        fe Zc, y;
        lds_load_fe(Zc, L.zc, lane);
        lds_load_fe(y, L.ys, lane);
        CurveK1::add(Q, P0, P1);
        FieldK1::mul(Zc, Zc, y);
        FieldK1::mul(Q.Z, Q.Z, Zc);
        coop_store_jac(L.pt[0], Q, lane);
    }
    __syncthreads();
    if (wave == 0 && active) {
        Jac Q, G, R;
        coop_load_jac(Q, L.pt[0], lane);
        coop_load_jac(G, L.pt[2], lane);
        CurveK1::add(R, Q, G);
        const bool ok = (flags & 3u) == 3u && !R.inf;
        Aff A;
        COOP_T(4);
        CurveK1::to_aff(A, R);
        COOP_T(5);
        FieldK1::normalize(A.x);
        FieldK1::normalize(A.y);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok) keccak_address(ad, A.x, A.y);
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = ad[q];
        status[i] = ok ? 0 : 1;
    }
    COOP_T(3);
}

// ------------------------------------------------------------------ cooperative kernel on fe26
// tx_verify_coop_kernel with the curve work of phases A and C on the 10 x 26-bit field (fe26.h): the
// same schedule, the same wave roles and the same pair split of every doubling and mixed addition, but
// a lone wave (one per SIMD here) no longer waits on carry chains: its field additions are independent
// limb adds and its multiplies are two interleaved mad chains.  Field elements cross between the two
// waves of a pair as their raw limbs (magnitudes travel with them, as the formulas state); the tables
// and phase results in LDS stay canonical 8-word values, so phase D is tx_verify_coop_kernel's.
// Bit-identical to tx_verify_kernel<0, *>.
struct Coop26Lds {
    uint32_t tab[8][16][64];          // co-Z table on E', canonical words: [entry][x0..7, y0..7][lane]
    uint32_t zc[8][64];
    uint32_t k[2][4][64];             // GLV halves
    uint32_t flags[64];               // bit0 scalars ok, bit1 R ok, bit2 neg1, bit3 neg2
    uint2 ex[2][2][6][5][64];         // [chain][writer role][slot][limb pair][lane]: one fe26 = 5 ds_write_b64
    uint32_t tabphx[8][8][64];        // beta * x of the table entries
    uint32_t pt[5][25][64];           // chain results 0/1, G partials 2..4 (canonical X, Y, Z, inf)
    uint32_t xe[8][64];
    uint32_t xrinv[8][64];
    uint32_t ys[8][64];
    uint32_t rflag[64];
    uint32_t post[2];
};

struct Coop26Ctx {
    Coop26Lds* L;
    int chain, role, lane;
    bool probe;  // BCOSGPU_COOP_TIMING
    __device__ __forceinline__ void puts(int s, const fe26& a) const {
        uint2* p = &L->ex[chain][role][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) p[q * 64] = make_uint2(a.v[2 * q], a.v[2 * q + 1]);
    }
    __device__ __forceinline__ void gets(int s, fe26& a) const {
        const uint2* p = &L->ex[chain][role ^ 1][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint2 w = p[q * 64];
            a.v[2 * q] = w.x;
            a.v[2 * q + 1] = w.y;
        }
    }
};

// as coop_dbl (slot buffers 0-2 / 3-5 alternate the same way); magnitudes as CurveK1x::dbl:
//   a: A = X^2, E = 3A (3), F = E^2, Z3 = 2 Y Z (2) | b: B = Y^2, D = 4 X B (4), C8 = 8 B^2 (8)
//   -> both: X3 = F - 2D (10), Y3 = E (D - X3) - C8 (10)
template <int S0>
__device__ __forceinline__ void coop26_dbl(Jac26& P, const Coop26Ctx& c) {
    fe26 E, F, D, C8, Z3, X3, Y3, t;
    DBL_T(0);
    if (c.role == 0) {
        fe26 A;
        fe26_sqr(A, P.X);
        fe26_mul_int<3>(E, A);
        fe26_sqr(F, E);
        c.puts(S0, E);
        c.puts(S0 + 1, F);
        fe26_mul(Z3, P.Y, P.Z);
        fe26_mul_int<2>(Z3, Z3);
        c.puts(S0 + 2, Z3);
    } else {
        fe26 B, C;
        fe26_sqr(B, P.Y);
        fe26_mul(D, P.X, B);
        fe26_mul_int<4>(D, D);
        c.puts(S0, D);
        fe26_sqr(C, B);
        fe26_mul_int<8>(C8, C);
        c.puts(S0 + 1, C8);
    }
    DBL_T(1);
    __syncthreads();
    DBL_T(2);
    if (c.role == 0) {
        c.gets(S0, D);
        c.gets(S0 + 1, C8);
    } else {
        c.gets(S0, E);
        c.gets(S0 + 1, F);
        c.gets(S0 + 2, Z3);
    }
    fe26_mul_int<2>(t, D);
    fe26_sub<9>(X3, F, t);
    fe26_sub<11>(t, D, X3);
    fe26_mul(Y3, E, t);
    fe26_sub<9>(Y3, Y3, C8);
    DBL_T(3);
    fe26_copy(P.X, X3);
    fe26_copy(P.Y, Y3);
    fe26_copy(P.Z, Z3);
    DBL_T(4);
}

// as coop_madd, with CurveK1x::madd's arrangement (r = 2 rr, Z3 = 2 Z1 H):
//   both: Z1Z1 | a: U2, H (12), HH, Z3 (2) | b: S2, rr (12), R2 = 4 rr^2 (4)
//   -> a: J = H I | b: V = X1 I        (I = 4 HH)
//   -> a: rr (V - X3) | b: Y1 J        -> Y3 = 2 (a - b) (6);  X3 = R2 - J - 2V (9)
__device__ __forceinline__ void coop26_madd(Jac26& R, const Jac26& P, const Aff26& Q, const Coop26Ctx& c) {
    fe26 Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    fe26_sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        fe26_mul(u, Q.x, Z1Z1);
        fe26_sub<11>(H, u, P.X);
        fe26_sqr(HH, H);
        fe26_mul(Z3, P.Z, H);
        fe26_mul_int<2>(Z3, Z3);
        c.puts(0, H);
        c.puts(1, HH);
        c.puts(2, Z3);
    } else {
        fe26_mul(u, Q.y, P.Z);
        fe26_mul(u, u, Z1Z1);
        fe26_sub<11>(rr, u, P.Y);
        fe26_sqr(R2, rr);
        fe26_mul_int<4>(R2, R2);
        c.puts(0, rr);
        c.puts(1, R2);
    }
    __syncthreads();
    if (c.role == 0) {
        c.gets(0, rr);
        c.gets(1, R2);
    } else {
        c.gets(0, H);
        c.gets(1, HH);
        c.gets(2, Z3);
    }
    fe26_mul_int<4>(I, HH);
    if (c.role == 0) {
        fe26_mul(J, H, I);
        c.puts(3, J);
    } else {
        fe26_mul(V, P.X, I);
        c.puts(3, V);
    }
    __syncthreads();
    if (c.role == 0) c.gets(3, V);
    else c.gets(3, J);
    fe26_sub<2>(X3, R2, J);
    fe26_mul_int<2>(t, V);
    fe26_sub<3>(X3, X3, t);
    if (c.role == 0) {
        fe26_sub<10>(t, V, X3);
        fe26_mul(u, rr, t);
        c.puts(4, u);
    } else {
        fe26_mul(u, P.Y, J);
        c.puts(4, u);
    }
    __syncthreads();
    c.gets(4, t);
    if (c.role == 0) fe26_sub<2>(Y3, u, t);
    else fe26_sub<2>(Y3, t, u);
    fe26_mul_int<2>(Y3, Y3);
    const bool hz = fe26_is_zero(H) && !P.inf;
    const bool rz = fe26_is_zero(rr);
    Jac26 D;
    if (hz && rz) CurveK1x::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe26_copy(R.X, X3);
    fe26_copy(R.Y, Y3);
    fe26_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveK1x::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe26_copy(R.X, Q.x);
        fe26_copy(R.Y, Q.y);
        fe26_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void coop26_add_digit(Jac26& acc, const Coop26Ctx& c, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    const uint32_t* bx = phi ? &c.L->tabphx[0][0][0] + m * (8 * 64) + c.lane : base;
    Aff26 S;
    {
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x[k] = bx[k * 64];
            y[k] = base[(8 + k) * 64];
        }
        fe26_from_words(S.x, x);
        fe26_from_words(S.y, y);
    }
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    Jac26 R;
    coop26_madd(R, acc, S, c);
    CurveK1x::cmov(acc, R, d != 0);
}

// acc = u1 * G restricted to 8-bit comb windows [lo, hi)
__device__ __forceinline__ void comb_range26(Jac26& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo,
                                             int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    CurveK1x::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        Aff26 T;
        load_aff26(T, tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        Jac26 S;
        CurveK1x::madd(S, acc, T);
        CurveK1x::cmov(acc, S, b != 0u);
    }
}

// canonical 8-word coordinates into a phase-result slot (the layout coop_load_jac reads)
__device__ __forceinline__ void coop26_store_jac(uint32_t (*dst)[64], const Jac26& P, int lane) {
    fe X, Y, Z;
    fe26_to_fe(X, P.X);
    fe26_to_fe(Y, P.Y);
    fe26_to_fe(Z, P.Z);
    Jac J;
    fe_copy(J.X, X);
    fe_copy(J.Y, Y);
    fe_copy(J.Z, Z);
    J.inf = P.inf;
    coop_store_jac(dst, J, lane);
}
__device__ __forceinline__ void coop26_load_jac(Jac26& P, const uint32_t (*src)[64], int lane) {
    Jac J;
    coop_load_jac(J, src, lane);
    fe26_from_fe(P.X, J.X);
    fe26_from_fe(P.Y, J.Y);
    fe26_from_fe(P.Z, J.Z);
    P.inf = J.inf;
}
__device__ __forceinline__ void lds_load_fe26(fe26& a, const uint32_t (*src)[64], int lane) {
    fe w;
    lds_load_fe(w, src, lane);
    fe26_from_fe(a, w);
}
__device__ __forceinline__ void lds_store_fe26(uint32_t (*dst)[64], const fe26& a, int lane) {
    fe w;
    fe26_to_fe(w, a);
    lds_store_fe(dst, w, lane);
}

__global__ __launch_bounds__(256, 1) void tx_verify_coop26_kernel(const uint8_t* __restrict__ pre,
                                                                  const uint64_t* __restrict__ pre_off,
                                                                  const uint8_t* __restrict__ sig,
                                                                  const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                  const uint32_t* __restrict__ tab,
                                                                  uint8_t* __restrict__ txhash,
                                                                  uint8_t* __restrict__ sender,
                                                                  uint8_t* __restrict__ status) {
    __shared__ Coop26Lds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    COOP_T(0);
    uint64_t sa = 0, sb = 0, pa = 0, pb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
        pa = pre_off[i];
        pb = pre_off[i + 1];
    }
    const uint32_t slen = (sb - sa) > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(sb - sa);
    if (threadIdx.x == 0) {
        L.post[0] = 0u;
        L.post[1] = 0u;
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase A (as tx_verify_coop_kernel)
    fe r, s;
    uint32_t v = 0;
    bool ok = false;
    if (active) ok = parse_sig65(sig + sa, slen, r, s, v);
    else { fe_zero(r); fe_zero(s); }
    if (wave == 1 || wave == 2) {
        fe x;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        fe26 X, rhs, t, seven;
        fe26_from_fe(X, x);
        fe26_sqr(t, X);
        fe26_mul(rhs, t, X);
        fe26_set_small(seven, 7u);
        fe26_add(rhs, rhs, seven);  // w (m 2)
        if (wave == 2) {
            fe26 y, ny;
            fe26_sqrt_cand(y, rhs);
            fe26_sqr(t, y);
            fe26_sub<3>(t, t, rhs);
            okr = okr && fe26_is_zero(t);
            fe26_normalize(y);
            fe26_neg<2>(ny, y);
            fe26_normalize(ny);
            fe26_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            lds_store_fe26(L.ys, y, lane);
            L.rflag[lane] = okr ? 2u : 0u;
            COOP_T(6);
        } else {
            Aff26 R, A[8];
            fe26_mul(R.x, rhs, X);  // w x
            fe26_sqr(R.y, rhs);     // w^2
            fe26 Zc, beta;
            {
                Jac26 T[8];
                multiples8_26(T, R);
                coz_table26(A, Zc, T);
            }
            fe26_const(beta, kGlvBeta);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe26(L.tab[j], A[j].x, lane);
                lds_store_fe26(L.tab[j] + 8, A[j].y, lane);
                fe26 bx;
                fe26_mul(bx, A[j].x, beta);
                lds_store_fe26(L.tabphx[j], bx, lane);
            });
            lds_store_fe26(L.zc, Zc, lane);
            COOP_T(6);
        }
    }
    if (!ok) {
        fe_zero(r);
        r.v[0] = 1;
        fe_zero(s);
    }
    if (wave == 3) {
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            keccak256_msg(rd, len, d);
            store_digest(KECCAK256, txhash + 32 * i, d);
        }
        fe e;
        fe_from_be_words(e, d);
        reduce_once(e, ParamN1::M);
        lds_store_fe(L.xe, e, lane);
        coop_post(&L.post[1]);
        COOP_T(7);
    } else if (wave == 0) {
        fe rm, rinv;
        FieldN1::from_plain(rm, r);
        FieldInv<FieldN1>::inv(rinv, rm);
        lds_store_fe(L.xrinv, rinv, lane);
        coop_post(&L.post[0]);
        COOP_T(7);
    }
    if (wave != 2) {
        coop_wait(&L.post[0]);
        coop_wait(&L.post[1]);
        fe e, rinv, u1;
        lds_load_fe(e, L.xe, lane);
        lds_load_fe(rinv, L.xrinv, lane);
        FieldN1::mul(u1, e, rinv);
        FieldN1::neg(u1, u1);
        if (wave == 1) {
            fe u2, k1, k2;
            FieldN1::mul(u2, s, rinv);
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L.k[0][q][lane] = k1.v[q];
                L.k[1][q][lane] = k2.v[q];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
        constexpr int kCombW0 = 12, kCombW1 = 24;
        Jac26 G;
        const int lo = wave == 0 ? 0 : wave == 3 ? kCombW0 : kCombW1;
        const int hi = wave == 0 ? kCombW0 : wave == 3 ? kCombW1 : 32;
        comb_range26(G, u1, tab, lo, hi);
        coop26_store_jac(L.pt[wave == 0 ? 2 : wave == 3 ? 3 : 4], G, lane);
    }
    COOP_T(1);
    __syncthreads();
    // ---------------------------------------------------------------- phase C: two cooperative GLV chains
    const uint32_t flags = L.flags[lane] | L.rflag[lane];
    Coop26Ctx c{&L, wave >> 1, wave & 1, lane, false};
    fe k;
    fe_zero(k);
#pragma unroll
    for (int q = 0; q < 4; ++q) k.v[q] = L.k[c.chain][q][lane];
    const bool neg = c.chain == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
    const bool phi = c.chain == 1;
    Jac26 acc;
    CurveK1x::set_inf(acc);
    coop26_add_digit(acc, c, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
    for (int w = 31; w >= 0; --w) {
        coop26_dbl<0>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = blockIdx.x == 0 && w == 20;
#endif
        coop26_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = false;
        if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][5] = clock64();
#endif
        coop26_dbl<0>(acc, c);
        coop26_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][6] = clock64();
#endif
        coop26_add_digit(acc, c, booth_digit128(k), neg, phi);
#ifdef BCOSGPU_COOP_TIMING
        if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][7] = clock64();
#endif
    }
    COOP_T(2);
    if (c.role == 0) coop26_store_jac(L.pt[c.chain], acc, lane);
    __syncthreads();
    // ---------------------------------------------------------------- phase D (on fe26 as well)
    if (wave == 1) {  // G part: partials 0 + 1 + 2
        Jac26 G0, G1, T, U;
        coop26_load_jac(G0, L.pt[2], lane);
        coop26_load_jac(G1, L.pt[3], lane);
        CurveK1x::add(T, G0, G1);
        coop26_load_jac(G0, L.pt[4], lane);
        CurveK1x::add(U, T, G0);
        coop26_store_jac(L.pt[2], U, lane);
    } else if (wave == 0) {  // R part: co-Z curve -> E_w (Z * Zc) -> E (Z * y)
        Jac26 P0, P1, Q;
        coop26_load_jac(P0, L.pt[0], lane);
        coop26_load_jac(P1, L.pt[1], lane);
        fe26 Zc, y;
        lds_load_fe26(Zc, L.zc, lane);
        lds_load_fe26(y, L.ys, lane);
        CurveK1x::add(Q, P0, P1);
        fe26_mul(Zc, Zc, y);
        fe26_mul(Q.Z, Q.Z, Zc);
        coop26_store_jac(L.pt[0], Q, lane);
    }
    __syncthreads();
    if (wave == 0 && active) {
        Jac26 Q, G, R;
        coop26_load_jac(Q, L.pt[0], lane);
        coop26_load_jac(G, L.pt[2], lane);
        CurveK1x::add(R, Q, G);
        const bool ok2 = (flags & 3u) == 3u && !R.inf;
        COOP_T(4);
        fe z, zi, ax, ay;
        fe26_to_fe(z, R.Z);
        FieldInv<FieldK1>::inv(zi, z);
        COOP_T(5);
        fe26 zi26, zi2, zi3, X, Y;
        fe26_from_fe(zi26, zi);
        fe26_sqr(zi2, zi26);
        fe26_mul(X, R.X, zi2);
        fe26_mul(zi3, zi2, zi26);
        fe26_mul(Y, R.Y, zi3);
        fe26_to_fe(ax, X);
        fe26_to_fe(ay, Y);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok2) keccak_address(ad, ax, ay);
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = ad[q];
        status[i] = ok2 ? 0 : 1;
    }
    COOP_T(3);
}

// ------------------------------------------------------------------ SM2 small-batch (pair) tx verify
// Guomi chains verify blocks of C2 size (FastSM2Crypto, FastSM2Crypto.h:33-44).  SM2 has no efficient
// endomorphism, so t*P is ONE chain of 256 doublings and 65 mixed additions.  A 256-thread workgroup
// owns 64 txs:
//   waves 0, 1  build the affine table 1P..8P (wave 0), then run the t*P chain as a PAIR that splits
//               every a = -3 doubling and mixed addition by dependency level and trades field elements
//               through LDS, synchronised by per-wave LDS counters (not workgroup barriers, so the other
//               two waves are never held up):
//                 dbl  (3M + 5S):  a: delta = Z^2, alpha = 3(X - delta)(X + delta), alpha^2
//                                  b: gamma = Y^2, 4 beta = 4 X gamma, 8 gamma^2
//                                  -> a: Y3 = alpha (4 beta - X3) - 8 gamma^2 | b: Z3 = 2 Y Z  (4 of 8 M/S)
//                 madd (7M + 4S):  as tx_verify_coop_kernel's                                   (6 of 11)
//   wave 2      tx hash, e = SM3(Z_A || h), the on-curve check, the address SM3(pub), comb windows
//               0..15 of s*G, then the sum of both comb halves;
//   wave 3      comb windows 16..31 of s*G.
// Waves 2 and 3 finish long before the chain; one final barrier, then wave 0 adds s*G, compares
// projectively and writes the verdict.  Bit-identical to tx_verify_kernel<1, *>.
struct Sm2PairLds {
    uint32_t tab[8][16][64];   // affine 1P..8P (Montgomery): [entry][x0..7, y0..7][lane]
    uint4 ex[2][2][3][2][64];  // [parity][writer role][slot][quad][lane]
    uint32_t g[25][64];        // s*G, Jacobian + inf (wave 2)
    uint32_t gh[25][64];       // comb windows 16..31 (wave 3)
    uint32_t c[8][64];         // (r - e) mod n, plain (wave 2)
    uint32_t addr[5][64];      // right160(SM3(pub)) (wave 2)
    uint32_t ok2[64];          // wave 2's checks: pub on the curve
    uint32_t seq[4];           // pair counters of waves 0, 1; wave 3 done
};

// One pair of waves: each exchange writes the caller's slots of the current parity, publishes its
// sequence number, waits for the partner's, reads the partner's slots and flips parity.  A parity's
// slots are rewritten only after the partner has published the NEXT exchange, i.e. after it has read
// them.
struct PairCtx {
    Sm2PairLds* L;
    int role, lane;
    uint32_t seq;
    int par;
    __device__ __forceinline__ void put(int s, const fe& a) const {
        uint4* p = &L->ex[par][role][s][0][0] + lane;
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void get(int s, fe& a) const {
        const uint4* p = &L->ex[par][role ^ 1][s][0][0] + lane;
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
    __device__ __forceinline__ void sync() {
        ++seq;
        __hip_atomic_store(&L->seq[role], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&L->seq[role ^ 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq) {
        }
    }
    __device__ __forceinline__ void next() { par ^= 1; }
};

// P = 2 P on SM2 (a = -3, dbl-2001-b with Z3 = 2 Y Z), P replicated on both waves of the pair
__device__ __forceinline__ void pair_dbl_am3(Jac& P, PairCtx& c) {
    using F = FieldP2;
    fe alpha, A2, b4, g8, X3, Y3, Z3, t, u;
    if (c.role == 0) {
        fe d;
        F::sqr(d, P.Z);
        F::sub(t, P.X, d);
        F::add(u, P.X, d);
        F::mul(alpha, t, u);
        F::mul3(alpha, alpha);
        F::sqr(A2, alpha);
        c.put(0, alpha);
        c.put(1, A2);
    } else {
        fe g;
        F::sqr(g, P.Y);
        F::mul(b4, P.X, g);
        F::template shl<2>(b4, b4);
        F::sqr(g8, g);
        F::template shl<3>(g8, g8);
        c.put(0, b4);
        c.put(1, g8);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, b4);
        c.get(1, g8);
    } else {
        c.get(0, alpha);
        c.get(1, A2);
    }
    c.next();
    F::template shl<1>(t, b4);
    F::sub(X3, A2, t);  // alpha^2 - 8 beta
    if (c.role == 0) {
        F::sub(t, b4, X3);
        F::mul(Y3, alpha, t);
        F::sub(Y3, Y3, g8);
        c.put(0, Y3);
    } else {
        F::mul(Z3, P.Y, P.Z);
        F::template shl<1>(Z3, Z3);
        c.put(0, Z3);
    }
    c.sync();
    if (c.role == 0) c.get(0, Z3);
    else c.get(0, Y3);
    c.next();
    fe_copy(P.X, X3);
    fe_copy(P.Y, Y3);
    fe_copy(P.Z, Z3);
}

// R = P + Q (madd-2007-bl with the complete-addition special cases of Curve::madd), Q affine
template <class F, class C>
__device__ __forceinline__ void pair_madd(Jac& R, const Jac& P, const Aff& Q, PairCtx& c) {
    fe Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    F::sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        F::mul(u, Q.x, Z1Z1);  // U2
        F::sub(H, u, P.X);
        F::sqr(HH, H);
        F::add(t, P.Z, H);
        F::sqr(Z3, t);
        F::sub(Z3, Z3, Z1Z1);
        F::sub(Z3, Z3, HH);
        c.put(0, H);
        c.put(1, HH);
        c.put(2, Z3);
    } else {
        F::mul(u, Q.y, P.Z);
        F::mul(u, u, Z1Z1);  // S2
        F::sub(rr, u, P.Y);
        F::template shl<1>(rr, rr);
        F::sqr(R2, rr);
        c.put(0, rr);
        c.put(1, R2);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, rr);
        c.get(1, R2);
    } else {
        c.get(0, H);
        c.get(1, HH);
        c.get(2, Z3);
    }
    c.next();
    F::template shl<2>(I, HH);
    if (c.role == 0) {
        F::mul(J, H, I);
        c.put(0, J);
    } else {
        F::mul(V, P.X, I);
        c.put(0, V);
    }
    c.sync();
    if (c.role == 0) c.get(0, V);
    else c.get(0, J);
    c.next();
    F::sub(X3, R2, J);
    F::template shl<1>(t, V);
    F::sub(X3, X3, t);
    if (c.role == 0) {
        F::sub(t, V, X3);
        F::mul(u, rr, t);  // rr (V - X3)
    } else {
        F::mul(u, P.Y, J);
        F::template shl<1>(u, u);  // 2 Y J
    }
    c.put(0, u);
    c.sync();
    c.get(0, t);
    c.next();
    if (c.role == 0) F::sub(Y3, u, t);
    else F::sub(Y3, t, u);
    // special cases, as Curve::madd (computed identically on both waves, no exchanges)
    const bool hz = F::is_zero(H) && !P.inf;
    const bool rz = F::is_zero(rr);
    Jac D;
    if (hz && rz) C::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe_copy(R.X, X3);
    fe_copy(R.Y, Y3);
    fe_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) C::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe_copy(R.X, Q.x);
        fe_copy(R.Y, Q.y);
        F::set_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void pair_add_digit_sm2(Jac& acc, PairCtx& c, int d) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = base[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    fe ny;
    FieldP2::neg(ny, S.y);
    fe_cmov(S.y, ny, d < 0);
    Jac R;
    pair_madd<FieldP2, CurveSM2>(R, acc, S, c);
    CurveSM2::cmov(acc, R, d != 0);
}

// acc = k * G restricted to the 8-bit comb windows [lo, hi)
template <class C>
__device__ __forceinline__ void comb_range8(Jac& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo,
                                            int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    C::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        Aff T;
        load_aff16(T, tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        Jac S;
        C::madd(S, acc, T);
        C::cmov(acc, S, b != 0u);
    }
}

__device__ __forceinline__ void pair_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = P.X.v[k];
        dst[8 + k][lane] = P.Y.v[k];
        dst[16 + k][lane] = P.Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void pair_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        P.X.v[k] = src[k][lane];
        P.Y.v[k] = src[8 + k][lane];
        P.Z.v[k] = src[16 + k][lane];
    }
    P.inf = src[24][lane] != 0u;
}

__global__ __launch_bounds__(256, 1) void tx_verify_sm2_pair_kernel(const uint8_t* __restrict__ pre,
                                                                    const uint64_t* __restrict__ pre_off,
                                                                    const uint8_t* __restrict__ sig,
                                                                    const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                    const uint32_t* __restrict__ tab,
                                                                    uint8_t* __restrict__ txhash,
                                                                    uint8_t* __restrict__ sender,
                                                                    uint8_t* __restrict__ status) {
    __shared__ Sm2PairLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    if (threadIdx.x < 4) L.seq[threadIdx.x] = 0u;
    __syncthreads();
    // signature r || s || pub (SM2Crypto::recover, SignatureDataWithPub.h:55-64); sm2_do_verify checks
    uint64_t sa = 0, sb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
    }
    const bool len_ok = active && sb - sa == 128u;
    fe r, s, px, py;
    uint32_t X[8], Y[8];
    if (len_ok) {
        ByteReader rd(sig + sa, 128);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(k);
        fe_from_be_words(r, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(8 + k);
        fe_from_be_words(s, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            X[k] = bswap32(rd.word(16 + k));
            Y[k] = bswap32(rd.word(24 + k));
        }
    } else {
        fe_zero(r);
        fe_zero(s);
#pragma unroll
        for (int k = 0; k < 8; ++k) X[k] = Y[k] = 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px.v[k] = X[7 - k];
        py.v[k] = Y[7 - k];
    }
    bool ok = len_ok && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    Aff P;
    FieldP2::from_plain(P.x, px);
    FieldP2::from_plain(P.y, py);
    Jac acc;
    if (wave <= 1) {
        PairCtx c{&L, wave, lane, 0u, 0};
        if (wave == 0) {
            Aff A[8];
            sm2_affine_table(A, P);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
            });
        }
        c.sync();  // the table is in LDS
        fe k;
        fe_copy(k, t);
        CurveSM2::set_inf(acc);
        pair_add_digit_sm2(acc, c, static_cast<int>(k.v[7] >> 31));  // digit 64 = bit 255
#pragma unroll 1
        for (int w = 63; w >= 0; --w) {
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
            const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            pair_add_digit_sm2(acc, c, d);
        }
    } else if (wave == 2) {
        // tx hash (TarsHashable.h:16-41), e = SM3(Z_A || h) (fast_sm2.cpp:34,203), c = (r - e) mod n
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint64_t pa = pre_off[i], pb = pre_off[i + 1];
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            sm3_msg(rd, len, d);
            store_digest(SM3, txhash + 32 * i, d);
        }
        fe h;
#pragma unroll
        for (int k = 0; k < 8; ++k) h.v[k] = d[7 - k];
        uint32_t eb[8];
        sm2_e(eb, X, Y, h);
        fe e, cc;
#pragma unroll
        for (int k = 0; k < 8; ++k) e.v[k] = eb[7 - k];
        reduce_once(e, ParamN2::M);
        FieldN2::sub(cc, r, e);
        lds_store_fe(L.c, cc, lane);
        fe b;
        fe_set(b, kSM2B);
        L.ok2[lane] = CurveSM2::on_curve(P, b) ? 1u : 0u;
        uint32_t ad[5];
        sm3_address(ad, px, py);
#pragma unroll
        for (int k = 0; k < 5; ++k) L.addr[k][lane] = ad[k];
        Jac G0, G1, G;
        comb_range8<CurveSM2>(G0, s, tab, 0, 16);
        while (__hip_atomic_load(&L.seq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
            __builtin_amdgcn_s_sleep(1);
        }
        pair_load_jac(G1, L.gh, lane);
        CurveSM2::add(G, G0, G1);
        pair_store_jac(L.g, G, lane);
    } else {
        Jac G1;
        comb_range8<CurveSM2>(G1, s, tab, 16, 32);
        pair_store_jac(L.gh, G1, lane);
        __hip_atomic_store(&L.seq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (wave == 0 && active) {
        Jac G, Q;
        pair_load_jac(G, L.g, lane);
        CurveSM2::add(Q, G, acc);
        ok = ok && L.ok2[lane] != 0u && !Q.inf;
        // x1 = X / Z^2 must be congruent to r - e (mod n): x1 = c or c + n (when c + n < p)
        fe cc, c2, cm, z2, rhs;
        lds_load_fe(cc, L.c, lane);
        FieldP2::sqr(z2, Q.Z);
        FieldP2::from_plain(cm, cc);
        FieldP2::mul(rhs, cm, z2);
        bool match = FieldP2::eq(rhs, Q.X);
        const uint32_t carry = fe_add_k(c2, cc, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            FieldP2::from_plain(cm, c2);
            FieldP2::mul(rhs, cm, z2);
            match = match || FieldP2::eq(rhs, Q.X);
        }
        ok = ok && match;
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ok ? L.addr[k][lane] : 0u;
        status[i] = ok ? 0 : 1;
    }
}

// ------------------------------------------------------------------ SM2 pair kernel on fp26
// tx_verify_sm2_pair_kernel with the t*P chain, the comb halves and the final check on fp26 (R' =
// 2^286, ecp26.h); the split of each doubling / mixed addition between the pair is the same, with the
// magnitude plan of CurveSM2x (each wave of the pair normalises the same operands, so both hold
// identical limbs).  Exchanged elements are 5 x uint2 (raw limbs, no canonicalisation).
struct Sm2Pair26Lds {
    uint32_t tab[8][16][64];         // affine 1P..8P in the R' domain, canonical words
    uint2 ex[2][2][3][5][64];        // [parity][writer role][slot][limb pair][lane]
    uint32_t g[25][64];
    uint32_t gh[25][64];
    uint32_t c[8][64];
    uint32_t addr[5][64];
    uint32_t ok2[64];
    uint32_t seq[4];
};

struct Pair26Ctx {
    Sm2Pair26Lds* L;
    int role, lane;
    uint32_t seq;
    int par;
    __device__ __forceinline__ void put(int s, const fp26& a) const {
        uint2* p = &L->ex[par][role][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) p[q * 64] = make_uint2(a.v[2 * q], a.v[2 * q + 1]);
    }
    __device__ __forceinline__ void get(int s, fp26& a) const {
        const uint2* p = &L->ex[par][role ^ 1][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint2 w = p[q * 64];
            a.v[2 * q] = w.x;
            a.v[2 * q + 1] = w.y;
        }
    }
    __device__ __forceinline__ void sync() {
        ++seq;
        __hip_atomic_store(&L->seq[role], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&L->seq[role ^ 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq) {
        }
    }
    __device__ __forceinline__ void next() { par ^= 1; }
};

// as pair_dbl_am3 with CurveSM2x::dbl's magnitudes (X <= 5, Y, Z <= 8 -> (2, 2, 2)):
//   a: alpha = 3 (X - d)(X + d) (3), alpha^2 (1) | b: 4 beta (4), 8 gamma^2 (8)
//   -> both: X3 = alpha^2 - 8 beta (2) -> a: Y3 (2) | b: Z3 = 2 Y Z (2)
__device__ __forceinline__ void pair26_dbl(JacP26& P, Pair26Ctx& c) {
    fp26 alpha, A2, b4, g8, X3, Y3, Z3, t, u;
    if (c.role == 0) {
        fp26 d;
        fp26_sqr(d, P.Z);
        fp26_sub<2>(t, P.X, d);
        fp26_add(u, P.X, d);
        fp26_mul(alpha, t, u);
        fp26_mul_int<3>(alpha, alpha);
        fp26_sqr(A2, alpha);
        c.put(0, alpha);
        c.put(1, A2);
    } else {
        fp26 g;
        fp26_sqr(g, P.Y);
        fp26_mul(b4, P.X, g);
        fp26_mul_int<4>(b4, b4);
        fp26_sqr(g8, g);
        fp26_mul_int<8>(g8, g8);
        c.put(0, b4);
        c.put(1, g8);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, b4);
        c.get(1, g8);
    } else {
        c.get(0, alpha);
        c.get(1, A2);
    }
    c.next();
    F26_SETM(alpha, 3);
    F26_SETM(A2, 1);
    F26_SETM(b4, 4);
    F26_SETM(g8, 8);
    fp26_mul_int<2>(t, b4);
    fp26_sub<9>(X3, A2, t);
    fp26_normalize_weak(X3);
    if (c.role == 0) {
        fp26_sub<3>(t, b4, X3);
        fp26_mul(Y3, alpha, t);
        fp26_sub<9>(Y3, Y3, g8);
        fp26_normalize_weak(Y3);
        c.put(0, Y3);
    } else {
        fp26_mul(Z3, P.Y, P.Z);
        fp26_mul_int<2>(Z3, Z3);
        c.put(0, Z3);
    }
    c.sync();
    if (c.role == 0) c.get(0, Z3);
    else c.get(0, Y3);
    c.next();
    F26_SETM(Y3, 2);
    F26_SETM(Z3, 2);
    fp26_copy(P.X, X3);
    fp26_copy(P.Y, Y3);
    fp26_copy(P.Z, Z3);
}

// as pair_madd with CurveSM2x::madd's arrangement (r = 2 rr, Z3 = 2 Z1 H): P (2, 2, <= 8), Q <= 2
//   a: H (5), HH, Z3 (2) | b: rr (5), R2 = 4 rr^2 (4) -> a: J | b: V -> a: rr (V - X3) | b: Y1 J
__device__ __forceinline__ void pair26_madd(JacP26& R, const JacP26& P, const AffP26& Q, Pair26Ctx& c) {
    fp26 Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    fp26_sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        fp26_mul(u, Q.x, Z1Z1);
        fp26_sub<3>(H, u, P.X);
        fp26_sqr(HH, H);
        fp26_mul(Z3, P.Z, H);
        fp26_mul_int<2>(Z3, Z3);
        c.put(0, H);
        c.put(1, HH);
        c.put(2, Z3);
    } else {
        fp26_mul(u, Q.y, P.Z);
        fp26_mul(u, u, Z1Z1);
        fp26_sub<3>(rr, u, P.Y);
        fp26_sqr(R2, rr);
        fp26_mul_int<4>(R2, R2);
        c.put(0, rr);
        c.put(1, R2);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, rr);
        c.get(1, R2);
    } else {
        c.get(0, H);
        c.get(1, HH);
        c.get(2, Z3);
    }
    c.next();
    F26_SETM(rr, 5);
    F26_SETM(R2, 4);
    F26_SETM(H, 5);
    F26_SETM(HH, 1);
    F26_SETM(Z3, 2);
    fp26_mul_int<4>(I, HH);
    if (c.role == 0) {
        fp26_mul(J, H, I);
        c.put(0, J);
    } else {
        fp26_mul(V, P.X, I);
        c.put(0, V);
    }
    c.sync();
    if (c.role == 0) c.get(0, V);
    else c.get(0, J);
    c.next();
    F26_SETM(V, 1);
    F26_SETM(J, 1);
    fp26_sub<2>(X3, R2, J);
    fp26_mul_int<2>(t, V);
    fp26_sub<3>(X3, X3, t);
    fp26_normalize_weak(X3);
    if (c.role == 0) {
        fp26_sub<3>(t, V, X3);
        fp26_mul(u, rr, t);
    } else {
        fp26_mul(u, P.Y, J);
    }
    c.put(0, u);
    c.sync();
    c.get(0, t);
    c.next();
    F26_SETM(t, 1);
    if (c.role == 0) fp26_sub<2>(Y3, u, t);
    else fp26_sub<2>(Y3, t, u);
    fp26_mul_int<2>(Y3, Y3);
    fp26_normalize_weak(Y3);
    const bool hz = fp26_is_zero(H) && !P.inf;
    const bool rz = fp26_is_zero(rr);
    JacP26 D;
    if (hz && rz) CurveSM2x::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fp26_copy(R.X, X3);
    fp26_copy(R.Y, Y3);
    fp26_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveSM2x::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fp26_copy(R.X, Q.x);
        fp26_copy(R.Y, Q.y);
        fp26_set(R.Z, p26::ONE_R);
        R.inf = false;
    }
}

__device__ __forceinline__ void pair26_add_digit(JacP26& acc, Pair26Ctx& c, int d) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    AffP26 S;
    {
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x[k] = base[k * 64];
            y[k] = base[(8 + k) * 64];
        }
        fp26_from_words(S.x, x);
        fp26_from_words(S.y, y);
    }
    fp26 ny;
    fp26_neg<2>(ny, S.y);
    fp26_cmov(S.y, ny, d < 0);
    fp26_normalize_weak(S.y);
    JacP26 R;
    pair26_madd(R, acc, S, c);
    CurveSM2x::cmov(acc, R, d != 0);
}

// acc = k * G restricted to the 8-bit comb windows [lo, hi) of the R'-domain table
__device__ __forceinline__ void comb_range_sm2_26(JacP26& acc, const fe& k_plain, const uint32_t* __restrict__ tab,
                                                  int lo, int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    CurveSM2x::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        AffP26 T;
        load_affp26(T, tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        JacP26 S;
        CurveSM2x::madd(S, acc, T);
        CurveSM2x::cmov(acc, S, b != 0u);
    }
}

__device__ __forceinline__ void pair26_store_jac(uint32_t (*dst)[64], const JacP26& P, int lane) {
    fe X, Y, Z;
    fp26_to_fe(X, P.X);
    fp26_to_fe(Y, P.Y);
    fp26_to_fe(Z, P.Z);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = X.v[k];
        dst[8 + k][lane] = Y.v[k];
        dst[16 + k][lane] = Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void pair26_load_jac(JacP26& P, const uint32_t (*src)[64], int lane) {
    uint32_t x[8], y[8], z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[k] = src[k][lane];
        y[k] = src[8 + k][lane];
        z[k] = src[16 + k][lane];
    }
    fp26_from_words(P.X, x);
    fp26_from_words(P.Y, y);
    fp26_from_words(P.Z, z);
    P.inf = src[24][lane] != 0u;
}

__global__ __launch_bounds__(256, 1) void tx_verify_sm2_pair26_kernel(const uint8_t* __restrict__ pre,
                                                                      const uint64_t* __restrict__ pre_off,
                                                                      const uint8_t* __restrict__ sig,
                                                                      const uint64_t* __restrict__ sig_off,
                                                                      uint64_t n, const uint32_t* __restrict__ tab,
                                                                      uint8_t* __restrict__ txhash,
                                                                      uint8_t* __restrict__ sender,
                                                                      uint8_t* __restrict__ status) {
    __shared__ Sm2Pair26Lds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    if (threadIdx.x < 4) L.seq[threadIdx.x] = 0u;
    __syncthreads();
    uint64_t sa = 0, sb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
    }
    const bool len_ok = active && sb - sa == 128u;
    fe r, s, px, py;
    uint32_t X[8], Y[8];
    if (len_ok) {
        ByteReader rd(sig + sa, 128);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(k);
        fe_from_be_words(r, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(8 + k);
        fe_from_be_words(s, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            X[k] = bswap32(rd.word(16 + k));
            Y[k] = bswap32(rd.word(24 + k));
        }
    } else {
        fe_zero(r);
        fe_zero(s);
#pragma unroll
        for (int k = 0; k < 8; ++k) X[k] = Y[k] = 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px.v[k] = X[7 - k];
        py.v[k] = Y[7 - k];
    }
    bool ok = len_ok && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    AffP26 P;
    fp26_from_plain(P.x, px);
    fp26_from_plain(P.y, py);
    JacP26 acc;
    if (wave <= 1) {
        Pair26Ctx c{&L, wave, lane, 0u, 0};
        if (wave == 0) {
            AffP26 A[8];
            sm2_affine_table26(A, P);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                fe x, y;
                fp26_to_fe(x, A[j].x);
                fp26_to_fe(y, A[j].y);
                lds_store_fe(L.tab[j], x, lane);
                lds_store_fe(L.tab[j] + 8, y, lane);
            });
        }
        c.sync();  // the table is in LDS
        fe k;
        fe_copy(k, t);
        CurveSM2x::set_inf(acc);
        pair26_add_digit(acc, c, static_cast<int>(k.v[7] >> 31));  // digit 64 = bit 255
#pragma unroll 1
        for (int w = 63; w >= 0; --w) {
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
            const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            pair26_add_digit(acc, c, d);
        }
    } else if (wave == 2) {
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint64_t pa = pre_off[i], pb = pre_off[i + 1];
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            sm3_msg(rd, len, d);
            store_digest(SM3, txhash + 32 * i, d);
        }
        fe h;
#pragma unroll
        for (int k = 0; k < 8; ++k) h.v[k] = d[7 - k];
        uint32_t eb[8];
        sm2_e(eb, X, Y, h);
        fe e, cc;
#pragma unroll
        for (int k = 0; k < 8; ++k) e.v[k] = eb[7 - k];
        reduce_once(e, ParamN2::M);
        FieldN2::sub(cc, r, e);
        lds_store_fe(L.c, cc, lane);
        L.ok2[lane] = sm2_on_curve26(P) ? 1u : 0u;
        uint32_t ad[5];
        sm3_address(ad, px, py);
#pragma unroll
        for (int k = 0; k < 5; ++k) L.addr[k][lane] = ad[k];
        JacP26 G0, G1, G;
        comb_range_sm2_26(G0, s, tab, 0, 16);
        while (__hip_atomic_load(&L.seq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
            __builtin_amdgcn_s_sleep(1);
        }
        pair26_load_jac(G1, L.gh, lane);
        CurveSM2x::add(G, G0, G1);
        pair26_store_jac(L.g, G, lane);
    } else {
        JacP26 G1;
        comb_range_sm2_26(G1, s, tab, 16, 32);
        pair26_store_jac(L.gh, G1, lane);
        __hip_atomic_store(&L.seq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (wave == 0 && active) {
        JacP26 G, Q;
        pair26_load_jac(G, L.g, lane);
        CurveSM2x::add(Q, G, acc);
        ok = ok && L.ok2[lane] != 0u && !Q.inf;
        fe cc, c2;
        lds_load_fe(cc, L.c, lane);
        fp26 z2, cm, rhs, dlt;
        fp26_sqr(z2, Q.Z);
        fp26_from_plain(cm, cc);
        fp26_mul(rhs, cm, z2);
        fp26_sub<3>(dlt, rhs, Q.X);
        bool match = fp26_is_zero(dlt);
        const uint32_t carry = fe_add_k(c2, cc, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            fp26_from_plain(cm, c2);
            fp26_mul(rhs, cm, z2);
            fp26_sub<3>(dlt, rhs, Q.X);
            match = match || fp26_is_zero(dlt);
        }
        ok = ok && match;
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ok ? L.addr[k][lane] : 0u;
        status[i] = ok ? 0 : 1;
    }
}

// ------------------------------------------------------------------ launchers
static inline unsigned grid_of(uint64_t n) { return static_cast<unsigned>((n + 255) / 256); }

int launch_secp256k1_recover(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride, uint64_t n,
                             uint8_t* d_pub, uint8_t* d_addr, uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    if (g_policy.f26)
        hipLaunchKernelGGL(secp256k1_recover_kernel<true>, dim3(grid_of(n)), dim3(256), 0, st, d_hash, d_sig, stride, n,
                           k1, bits, d_pub, d_addr, d_ok);
    else
        hipLaunchKernelGGL(secp256k1_recover_kernel<false>, dim3(grid_of(n)), dim3(256), 0, st, d_hash, d_sig, stride, n,
                           k1, bits, d_pub, d_addr, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_sm2_verify(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride, uint64_t n, uint8_t* d_addr,
                      uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    if (g_policy.f26) {
        const uint32_t* t26;
        int b26;
        rc = tables_sm2_26(&t26, &b26);
        if (rc) return rc;
        hipLaunchKernelGGL(sm2_verify_kernel<true>, dim3(grid_of(n)), dim3(256), 0, st, d_hash, d_sig, stride, n, t26,
                           b26, d_addr, d_ok);
    } else {
        hipLaunchKernelGGL(sm2_verify_kernel<false>, dim3(grid_of(n)), dim3(256), 0, st, d_hash, d_sig, stride, n, sm2,
                           bits, d_addr, d_ok);
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
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

int launch_sig_verify(int suite, const uint8_t* d_pub, const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride,
                      uint64_t n, uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    if (suite == BCOSGPU_SUITE_SM2 && g_policy.f26) {
        const uint32_t* t26;
        int b26;
        rc = tables_sm2_26(&t26, &b26);
        if (rc) return rc;
        hipLaunchKernelGGL((sig_verify_kernel<BCOSGPU_SUITE_SM2, true>), dim3(grid_of(n)), dim3(256), 0, st, d_pub,
                           d_hash, d_sig, stride, n, t26, b26, d_ok);
    } else if (suite == BCOSGPU_SUITE_SM2)
        hipLaunchKernelGGL(sig_verify_kernel<BCOSGPU_SUITE_SM2>, dim3(grid_of(n)), dim3(256), 0, st, d_pub, d_hash, d_sig,
                           stride, n, sm2, bits, d_ok);
    else if (g_policy.f26)
        hipLaunchKernelGGL((sig_verify_kernel<BCOSGPU_SUITE_SECP256K1, true>), dim3(grid_of(n)), dim3(256), 0, st, d_pub,
                           d_hash, d_sig, stride, n, k1, bits, d_ok);
    else
        hipLaunchKernelGGL(sig_verify_kernel<BCOSGPU_SUITE_SECP256K1>, dim3(grid_of(n)), dim3(256), 0, st, d_pub, d_hash,
                           d_sig, stride, n, k1, bits, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_ecrecover(const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    if (g_policy.f26)
        hipLaunchKernelGGL(ecrecover_kernel<true>, dim3(grid_of(n)), dim3(256), 0, st, d_in, n, k1, bits, d_out, d_ok);
    else
        hipLaunchKernelGGL(ecrecover_kernel<false>, dim3(grid_of(n)), dim3(256), 0, st, d_in, n, k1, bits, d_out, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_tx_verify(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off, const uint8_t* d_sig,
                     const uint64_t* d_sig_off, uint64_t n, uint8_t* d_txhash, uint8_t* d_sender, uint8_t* d_status,
                     hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits;
    int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    const TxKernelPolicy pol = g_policy;
    // small secp256k1 batches (SIMDs left idle by one tx per lane): the cooperative-pair kernel
    // (C2), or the 4-wave split kernel; both on the L2-resident 8-bit comb tables
    const bool small = pol.split >= 0 ? pol.split == 1 : n <= (1ull << 15);
    if (suite == BCOSGPU_SUITE_SECP256K1 && small) {
        rc = tables8(&k1, &sm2);
        if (rc) return rc;
        const dim3 grid(static_cast<unsigned>((n + 63) / 64));
        if (pol.coop && pol.f26)
            hipLaunchKernelGGL(tx_verify_coop26_kernel, grid, dim3(256), 0, st, d_pre, d_pre_off, d_sig, d_sig_off, n,
                               k1, d_txhash, d_sender, d_status);
        else if (pol.coop)
            hipLaunchKernelGGL(tx_verify_coop_kernel, grid, dim3(256), 0, st, d_pre, d_pre_off, d_sig, d_sig_off, n, k1,
                               d_txhash, d_sender, d_status);
        else
            hipLaunchKernelGGL(tx_verify_split_kernel, grid, dim3(256), 0, st, d_pre, d_pre_off, d_sig, d_sig_off, n,
                               k1, d_txhash, d_sender, d_status);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
    if (suite == BCOSGPU_SUITE_SM2 && small && pol.coop && pol.f26) {  // the SM2 pair kernel on fp26
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_tab_sm2_26[dev]) return BCOSGPU_E_NODEV;
        hipLaunchKernelGGL(tx_verify_sm2_pair26_kernel, dim3(static_cast<unsigned>((n + 63) / 64)), dim3(256), 0, st,
                           d_pre, d_pre_off, d_sig, d_sig_off, n, g_tab_sm2_26[dev], d_txhash, d_sender, d_status);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
    if (suite == BCOSGPU_SUITE_SM2 && small && pol.coop) {  // the SM2 pair kernel (8-bit comb)
        rc = tables8(&k1, &sm2);
        if (rc) return rc;
        hipLaunchKernelGGL(tx_verify_sm2_pair_kernel, dim3(static_cast<unsigned>((n + 63) / 64)), dim3(256), 0, st,
                           d_pre, d_pre_off, d_sig, d_sig_off, n, sm2, d_txhash, d_sender, d_status);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
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
