// ecc_device.h -- device side of the ECC kernels (gfx950, one signature per lane, integer ALU only):
// curve constants, comb-table geometry, scalar multiplication, the one-lane recover / verify bodies,
// plus the host declarations the kernel TUs share (tables and policy live in ecc_tables.hip).
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
#pragma once
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

// per-lane field elements and points in LDS, [word][lane] (conflict-free)
__device__ __forceinline__ void lds_store_fe(uint32_t (*dst)[64], const fe& a, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k][lane] = a.v[k];
}
__device__ __forceinline__ void lds_load_fe(fe& a, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a.v[k] = src[k][lane];
}

// Kernel-selection policy, read from the environment once (at the first bcosgpu_init) and settable
// through bcosgpu_set_tx_kernel_policy (tests, tuning); never read per launch.
struct TxKernelPolicy {
    int split = -1;  // small-batch secp kernels: -1 by size (n <= 2^15), 0 never, 1 always
    int occ = 0;     // tx_verify_kernel occupancy: 0 by size (2 for n >= 2^17), 1 or 2 forced
    int coop = 2;    // small-batch secp kernel: 3 row kernel, 2 lane-trio (fe26 only), 1 cooperative-pair, 0 4-wave split
                     // (automatic policy: 2 = choose among row / trio / pair / one-lane by rounds x latency)
    int f26 = 1;     // throughput secp kernels: 1 point arithmetic on the 10 x 26-bit field, 0 on FieldK1
};

// host-side state (ecc_tables.hip); a snapshot taken under the policy lock
TxKernelPolicy tx_policy();
// The comb tables of the current device: the 16-bit ones when present (*bits = 16), else the 8-bit
// ones (*bits = 8).
int tables(const uint32_t** k1, const uint32_t** sm2, int* bits);
// the SM2 comb table in fp26's R' domain: the 16-bit one when present, else the 8-bit one
int tables_sm2_26(const uint32_t** tab, int* bits);
// 8-bit comb tables (and the 8-bit SM2 table in the R' domain)
int tables8(const uint32_t** k1, const uint32_t** sm2);
int tables8_sm2_26(const uint32_t** tab);
// small-batch verify launchers (ecc_coop.hip: secp256k1; ecc_pair.hip: SM2), instantiated for TxIO and
// SigIO (the I/O policies below); SigIO has the fe26 / fp26 lane-trio and pair kernels only
struct TxIO;
struct SigIO;
struct EcrecIO;
struct KeyIO;
template <class IO>
int launch_verify_small_secp(const TxKernelPolicy& pol, const IO& io, uint64_t n, hipStream_t st);
// secp256k1 verify with a known key (KeyIO) on the lane-trio kernel (ecc_coop.hip)
int launch_sig_verify_small_secp(const KeyIO& io, uint64_t n, hipStream_t st);
// secp256k1 recovery, one signature per workgroup on row-spread field elements (ecc_row.hip)
template <class IO>
int launch_recover_row(const IO& io, uint64_t n, hipStream_t st);
// secp256k1 verify with a known key, one signature per workgroup on the rows (ecc_row.hip)
int launch_sig_verify_row_secp(const KeyIO& io, uint64_t n, hipStream_t st);
// SM2 verify (TxIO, SigIO, KeyIO), one signature per workgroup on the rows (ecc_row.hip)
template <class IO>
int launch_sm2_verify_row(const IO& io, uint64_t n, hipStream_t st);
// SM2 verify with a known key over KeyIO (ecc_txv.hip: launch_verify's kernel choice)
int launch_sm2_verify_key(const uint8_t* d_pub, const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride,
                          uint64_t n, uint8_t* d_ok, hipStream_t st);
template <class IO>
int launch_verify_small_sm2(const TxKernelPolicy& pol, const IO& io, uint64_t n, hipStream_t st);
static inline unsigned grid_of(uint64_t n) { return static_cast<unsigned>((n + 255) / 256); }

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

// ------------------------------------------------------------------ kernel I/O policies
// parse r, s, v of a 65-byte signature; ok = libsecp256k1 parse_compact + r, s != 0 (r, s zero and
// v = 0 for any other length, so every later check fails too)
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
// r || s || X || Y of a 128-byte SM2 signature-with-key at p (X, Y as big-endian word arrays)
__device__ __forceinline__ void parse_sm2_128(const uint8_t* p, fe& r, fe& s, uint32_t X[8], uint32_t Y[8]) {
    ByteReader rd(p, 128);
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
}
__device__ __forceinline__ void zero_sm2_sig(fe& r, fe& s, uint32_t X[8], uint32_t Y[8]) {
    fe_zero(r);
    fe_zero(s);
#pragma unroll
    for (int k = 0; k < 8; ++k) X[k] = Y[k] = 0u;
}

// Every verification kernel body (one-lane, lane-trio, cooperative pair) is written once over one of:
//   TxIO  -- Transaction::verify (Transaction.h:68-82): the digest is H(preimage) and is an output
//            (txhash); signature i = sig[sig_off[i] .. sig_off[i+1]); results sender20 and status
//            (0 ok / 1 InvalidSignature).
//   SigIO -- SignatureCrypto::recover with the digest given (Secp256k1Crypto::recover,
//            Secp256k1Crypto.cpp:79-93; SM2Crypto::recover, SM2Crypto.cpp:81-92): 32-byte digests,
//            signatures at a fixed stride and length; results pub64 (secp256k1 only, nullable), addr20
//            (nullable) and ok (1 valid / 0 invalid).  Output rows need 4-byte alignment only.
//   EcrecIO -- the EVM ecRecover precompile (Precompiled.cpp:443-482): input hash || v || r || s (128 B,
//            recid = (byte)(in[63] - 27)), output 12 zero bytes || address and ok.
//   KeyIO -- SignatureCrypto::verify(pub, hash, sig) with a KNOWN key (Secp256k1Crypto.cpp:51-63,
//            SM2Crypto.cpp:66-79): digests given, r || s = the first 64 bytes at a stride, keys pub64;
//            result ok only.
// The signature comes out of the policy parsed: rsv (secp256k1 recover: r, s, v and the
// parse_compact verdict) or sm2_sig (r, s and the key X, Y; false when the signature is not
// well-formed, e.g. not 128 bytes).
struct TxIO {
    const uint8_t* pre;
    const uint64_t* pre_off;
    const uint8_t* sig;
    const uint64_t* sig_off;
    uint8_t* txhash;
    uint8_t* sender;
    uint8_t* status;

    __device__ __forceinline__ uint32_t sig_span(uint64_t i, const uint8_t*& p) const {
        const uint64_t a = sig_off[i], b = sig_off[i + 1];
        p = sig + a;
        return b - a > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(b - a);
    }
    __device__ __forceinline__ bool rsv(uint64_t i, fe& r, fe& s, uint32_t& v) const {
        const uint8_t* p;
        const uint32_t l = sig_span(i, p);
        return parse_sig65(p, l, r, s, v);
    }
    __device__ __forceinline__ bool sm2_sig(uint64_t i, fe& r, fe& s, uint32_t X[8], uint32_t Y[8]) const {
        const uint8_t* p;
        if (sig_span(i, p) != 128u) {
            zero_sm2_sig(r, s, X, Y);
            return false;
        }
        parse_sm2_128(p, r, s, X, Y);
        return true;
    }
    // the digest as the field element the recover / verify bodies take (hash_be)
    template <int H>
    __device__ __forceinline__ void digest(uint64_t i, fe& h) const {
        const uint64_t a = pre_off[i];
        const uint32_t len = static_cast<uint32_t>(pre_off[i + 1] - a);
        ByteReader rd(pre + a, len);
        uint32_t d[8];
        if constexpr (H == SM3) {
            sm3_msg(rd, len, d);
#pragma unroll
            for (int k = 0; k < 8; ++k) h.v[k] = d[7 - k];
        } else {
            keccak256_msg(rd, len, d);
            fe_from_be_words(h, d);
        }
        store_digest(H, txhash + 32 * i, d);
    }
    __device__ __forceinline__ bool want_addr() const { return true; }
    // ad = right160(H(pub)) as 5 memory words (zero when !ok); x, y = the recovered key (unused here)
    __device__ __forceinline__ void finish(uint64_t i, bool ok, const uint32_t ad[5], const fe*, const fe*) const {
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ad[k];
        status[i] = ok ? 0 : 1;
    }
};

struct SigIO {
    const uint8_t* hash;
    const uint8_t* sig;
    uint32_t stride;
    uint32_t siglen;
    uint8_t* pub;
    uint8_t* addr;
    uint8_t* ok;

    __device__ __forceinline__ uint32_t sig_span(uint64_t i, const uint8_t*& p) const {
        p = sig + static_cast<uint64_t>(stride) * i;
        return siglen;
    }
    __device__ __forceinline__ bool rsv(uint64_t i, fe& r, fe& s, uint32_t& v) const {
        return parse_sig65(sig + static_cast<uint64_t>(stride) * i, siglen, r, s, v);
    }
    __device__ __forceinline__ bool sm2_sig(uint64_t i, fe& r, fe& s, uint32_t X[8], uint32_t Y[8]) const {
        if (siglen != 128u) {
            zero_sm2_sig(r, s, X, Y);
            return false;
        }
        parse_sm2_128(sig + static_cast<uint64_t>(stride) * i, r, s, X, Y);
        return true;
    }
    template <int H>
    __device__ __forceinline__ void digest(uint64_t i, fe& h) const {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(hash + 32 * i);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = q[k];
        fe_from_be_words(h, w);
    }
    __device__ __forceinline__ bool want_addr() const { return addr != nullptr; }
    __device__ __forceinline__ void finish(uint64_t i, bool valid, const uint32_t ad[5], const fe* x, const fe* y) const {
        if (pub && x && y) {
            fe zx, zy;
            fe_zero(zx);
            fe_zero(zy);
            store_be256_u32(pub + 64 * i, valid ? *x : zx);
            store_be256_u32(pub + 64 * i + 32, valid ? *y : zy);
        }
        if (addr) {
            uint32_t* o = reinterpret_cast<uint32_t*>(addr + 20 * i);
#pragma unroll
            for (int k = 0; k < 5; ++k) o[k] = valid ? ad[k] : 0u;
        }
        ok[i] = valid ? 1 : 0;
    }
};

struct EcrecIO {
    const uint8_t* in;  // n x 128, 16-byte aligned
    uint8_t* out;       // n x 32
    uint8_t* ok;

    __device__ __forceinline__ bool rsv(uint64_t i, fe& r, fe& s, uint32_t& v) const {
        const uint8_t* p = in + 128 * i;
        load_be256_aligned(r, p + 64);
        load_be256_aligned(s, p + 96);
        v = ((reinterpret_cast<const uint32_t*>(p)[15] >> 24) - 27u) & 0xffu;  // (byte)(in[63] - 27)
        return v <= 3u && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, ParamN1::M);
    }
    template <int H>
    __device__ __forceinline__ void digest(uint64_t i, fe& h) const {
        load_be256_aligned(h, in + 128 * i);
    }
    __device__ __forceinline__ bool want_addr() const { return true; }
    __device__ __forceinline__ void finish(uint64_t i, bool valid, const uint32_t ad[5], const fe*, const fe*) const {
        uint32_t* o = reinterpret_cast<uint32_t*>(out + 32 * i);
#pragma unroll
        for (int k = 0; k < 3; ++k) o[k] = 0u;
#pragma unroll
        for (int k = 0; k < 5; ++k) o[3 + k] = valid ? ad[k] : 0u;
        ok[i] = valid ? 1 : 0;
    }
};

struct KeyIO {
    const uint8_t* pub;   // n x 64 (X || Y)
    const uint8_t* hash;  // n x 32
    const uint8_t* sig;   // item i at sig + stride i: r || s (only the first 64 bytes are read)
    uint32_t stride;
    uint8_t* ok;

    template <int H>
    __device__ __forceinline__ void digest(uint64_t i, fe& h) const {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(hash + 32 * i);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = q[k];
        fe_from_be_words(h, w);
    }
    // secp256k1: r, s and the key as plain words (x, y)
    __device__ __forceinline__ void key_rs(uint64_t i, fe& r, fe& s, fe& x, fe& y) const {
        ByteReader rs(sig + static_cast<uint64_t>(stride) * i, 64), rp(pub + 64 * i, 64);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rs.word(k);
        fe_from_be_words(r, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rs.word(8 + k);
        fe_from_be_words(s, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rp.word(k);
        fe_from_be_words(x, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rp.word(8 + k);
        fe_from_be_words(y, w);
    }
    // SM2: r || s from the signature, X || Y from the key array (SM2Crypto::verify, SM2Crypto.cpp:66-79)
    __device__ __forceinline__ bool sm2_sig(uint64_t i, fe& r, fe& s, uint32_t X[8], uint32_t Y[8]) const {
        ByteReader rs(sig + static_cast<uint64_t>(stride) * i, 64), rp(pub + 64 * i, 64);
        uint32_t w[8];
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
        return true;
    }
    __device__ __forceinline__ bool want_addr() const { return false; }
    __device__ __forceinline__ void finish(uint64_t i, bool valid, const uint32_t*, const fe*, const fe*) const {
        ok[i] = valid ? 1 : 0;
    }
};

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

}  // namespace bcosgpu
