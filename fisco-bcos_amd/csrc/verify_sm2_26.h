// verify_sm2_26.h -- SM2 verification with the point arithmetic over fp26 (fp26.h / ecp26.h,
// Montgomery R' = 2^286), for the SM2 throughput kernels.  Same decisions and outputs as sm2_verify_rs
// (sm2_do_verify semantics, SM2Crypto.cpp:66-92 -> fast_sm2.cpp:139-227): the scalar work (range
// checks, t = r + s mod n, e = SM3(Z_A || h)) stays 8 x 32-bit; t*P (table 1P..8P, 65 radix-16 Booth
// windows), s*G (comb over tables re-expressed in the R' domain at init) and the projective x-check run
// on fp26.  Included by ecc_device.h after its SM2 helpers.
#pragma once
#include "ecp26.h"

namespace bcosgpu {

__device__ __forceinline__ void fp26_from_fe(fp26& r, const fe& a) { fp26_from_words(r, a.v); }
__device__ __forceinline__ void fp26_to_fe(fe& r, const fp26& a) {  // canonical words of the stored value
    fp26 t;
    fp26_copy(t, a);
    fp26_normalize(t);
    fp26_to_words(r.v, t);
}
__device__ __forceinline__ void fp26_from_plain(fp26& r, const fe& a) {  // a < 2^256 plain -> a R' mod p
    fp26 t;
    fp26_from_fe(t, a);
    fp26_to_mont(r, t);
}

// z^-1 in the R' domain from z R': the plain inverse of the stored integer by safegcd, times R'^3
__device__ __forceinline__ void fp26_inv(fp26& r, const fp26& a) {
    fe w, wi;
    fp26_to_fe(w, a);
    modinv_safegcd(wi, w, kMod30P2);
    fp26 t, k;
    fp26_from_fe(t, wi);
    fp26_set(k, p26::R3);
    fp26_mul(r, t, k);
}

__device__ __forceinline__ void load_affp26(AffP26& T, const uint32_t* __restrict__ e32) {
    const uint4* e = reinterpret_cast<const uint4*>(e32);
    const uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
    const uint32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const uint32_t y[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    fp26_from_words(T.x, x);
    fp26_from_words(T.y, y);
}

// y^2 == x^3 - 3x + b for P in the R' domain (P.x, P.y <= 2)
__device__ __forceinline__ bool sm2_on_curve26(const AffP26& P) {
    fp26 l, rr, t, b;
    fp26_sqr(l, P.y);
    fp26_sqr(t, P.x);
    fp26_mul(rr, t, P.x);
    fp26_mul_int<3>(t, P.x);
    fp26_sub<4>(rr, rr, t);  // m 6
    fp26_set(b, p26::B_R);
    fp26_add(rr, rr, b);     // m 7
    fp26_sub<8>(l, l, rr);
    return fp26_is_zero(l);
}

// acc = k * G over a BITS-bit comb table in the R' domain
template <int BITS>
__device__ __forceinline__ void comb_mul_sm2_26(JacP26& acc, const fe& k_plain, const uint32_t* __restrict__ tab) {
    constexpr int W = 256 / BITS;
    constexpr uint32_t E = 1u << BITS, MASK = E - 1u;
    fe k;
    fe_copy(k, k_plain);
    CurveSM2x::set_inf(acc);
#pragma unroll 1
    for (int i = 0; i < W; ++i) {
        const uint32_t b = k.v[0] & MASK;
        shr_bits<BITS>(k);
        AffP26 T;
        load_affp26(T, tab + (static_cast<size_t>(i) * E + b) * 16);
        JacP26 S;
        CurveSM2x::madd(S, acc, T);
        CurveSM2x::cmov(acc, S, b != 0u);
    }
}
__device__ __forceinline__ void comb_mul_sm2_26_rt(JacP26& acc, const fe& k, CombTab tab) {
    if (tab.bits == kWideBits) comb_mul_sm2_26<kWideBits>(acc, k, tab.p);
    else comb_mul_sm2_26<8>(acc, k, tab.p);
}

// affine table 1P..8P (m = 1): multiples in Jacobian, one inversion over the product of the Z's
__device__ __forceinline__ void sm2_affine_table26(AffP26 A[8], const AffP26& P) {
    JacP26 T[8];
    CurveSM2x::from_aff(T[0], P);
    CurveSM2x::dbl(T[1], T[0]);
    CurveSM2x::madd(T[2], T[1], P);
    CurveSM2x::dbl(T[3], T[1]);
    CurveSM2x::madd(T[4], T[3], P);
    CurveSM2x::dbl(T[5], T[2]);
    CurveSM2x::madd(T[6], T[5], P);
    CurveSM2x::dbl(T[7], T[3]);
    fp26 pre[8], inv;
    fp26_set(pre[0], p26::ONE_R);
    Unroll<1, 8>::run([&](auto J) { fp26_mul(pre[J], pre[J - 1], T[J].Z); });
    fp26_inv(inv, pre[7]);  // (Z1 ... Z7)^-1
    fp26_copy(A[0].x, P.x);
    fp26_copy(A[0].y, P.y);
    Unroll<0, 7>::run([&](auto J) {
        constexpr int j = 7 - decltype(J)::value;
        fp26 zi, zi2, zi3;
        fp26_mul(zi, inv, pre[j - 1]);  // Z_j^-1
        fp26_mul(inv, inv, T[j].Z);     // (Z1 .. Z(j-1))^-1
        fp26_sqr(zi2, zi);
        fp26_mul(zi3, zi2, zi);
        fp26_mul(A[j].x, T[j].X, zi2);
        fp26_mul(A[j].y, T[j].Y, zi3);
    });
}

// acc += d P from the table (d in -8..8): x as canonical words in LDS ([entry][word][lane], ldsx offset
// by the lane) or registers, y as canonical words in registers
template <bool LDS>
__device__ __forceinline__ void add_digit_sm2_26(JacP26& acc, const uint32_t* ldsx, const fe X[8], const fe Y[8], int d) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    AffP26 S;
    fe x, y;
    if constexpr (LDS) {
        const uint32_t* b = ldsx + m * 512u;
#pragma unroll
        for (int k = 0; k < 8; ++k) x.v[k] = b[k * 64];
    } else {
        fe_copy(x, X[0]);
#pragma unroll
        for (int q = 1; q < 8; ++q) fe_cmov(x, X[q], m == static_cast<uint32_t>(q));
    }
    fe_copy(y, Y[0]);
#pragma unroll
    for (int q = 1; q < 8; ++q) fe_cmov(y, Y[q], m == static_cast<uint32_t>(q));
    fp26_from_fe(S.x, x);
    fp26_from_fe(S.y, y);
    fp26 ny;
    fp26_neg<2>(ny, S.y);
    fp26_cmov(S.y, ny, d < 0);  // m 3 (madd takes Q <= 11)
    JacP26 R;
    CurveSM2x::madd(R, acc, S);
    CurveSM2x::cmov(acc, R, d != 0);
}

template <bool LDS>
__device__ __forceinline__ void booth_mul_sm2_26(JacP26& acc, const fe& k_plain, const AffP26& P, uint32_t* ldsx) {
    fe X[8], Y[8];
    {
        AffP26 A[8];
        sm2_affine_table26(A, P);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            fe x;
            fp26_to_fe(x, A[j].x);
            if constexpr (LDS) {
#pragma unroll
                for (int w = 0; w < 8; ++w) ldsx[(j * 8 + w) * 64] = x.v[w];
            } else {
                fe_copy(X[j], x);
            }
            fp26_to_fe(Y[j], A[j].y);
        }
    }
    fe k;
    fe_copy(k, k_plain);
    CurveSM2x::set_inf(acc);
    add_digit_sm2_26<LDS>(acc, ldsx, X, Y, static_cast<int>(k.v[7] >> 31));  // digit 64
#pragma unroll 1
    for (int i = 63; i >= 0; --i) {
        CurveSM2x::dbl(acc, acc);
        CurveSM2x::dbl(acc, acc);
        CurveSM2x::dbl(acc, acc);
        CurveSM2x::dbl(acc, acc);
        const uint32_t top = k.v[7];
        const uint32_t W = top >> 28, c = (top >> 27) & 1u;
        const int d = static_cast<int>(W + c) - static_cast<int>((W >> 3) << 4);
        shl4(k);
        add_digit_sm2_26<LDS>(acc, ldsx, X, Y, d);
    }
}

// sm2_verify_rs on fp26 (same contract; `tab` is the R'-domain comb table)
template <bool LDS = false>
__device__ __forceinline__ bool sm2_verify_rs26(const fe& hash_be, const fe& r, const fe& s, const uint32_t X[8],
                                                const uint32_t Y[8], CombTab tab, fe& px, fe& py,
                                                uint32_t* ldsx = nullptr) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        px.v[i] = X[7 - i];
        py.v[i] = Y[7 - i];
    }
    bool ok = fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    AffP26 P;
    fp26_from_plain(P.x, px);
    fp26_from_plain(P.y, py);
    ok = ok && sm2_on_curve26(P);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    uint32_t eb[8];
    sm2_e(eb, X, Y, hash_be);
    fe e;
#pragma unroll
    for (int i = 0; i < 8; ++i) e.v[i] = eb[7 - i];
    reduce_once(e, ParamN2::M);
    JacP26 QG, QP, Q;
    booth_mul_sm2_26<LDS>(QP, t, P, ldsx);
    comb_mul_sm2_26_rt(QG, s, tab);
    CurveSM2x::add(Q, QG, QP);
    ok = ok && !Q.inf;
    // x1 = X / Z^2 must be congruent to r - e (mod n): x1 = c or c + n (when c + n < p)
    fe c, c2;
    FieldN2::sub(c, r, e);
    fp26 z2, cm, rhs, dlt;
    fp26_sqr(z2, Q.Z);
    fp26_from_plain(cm, c);
    fp26_mul(rhs, cm, z2);
    fp26_sub<13>(dlt, rhs, Q.X);  // Q.X <= 12 (CurveSM2x::add)
    bool match = fp26_is_zero(dlt);
    const uint32_t carry = fe_add_k(c2, c, ParamN2::M);
    if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
        fp26_from_plain(cm, c2);
        fp26_mul(rhs, cm, z2);
        fp26_sub<13>(dlt, rhs, Q.X);
        match = match || fp26_is_zero(dlt);
    }
    return ok && match;
}

template <bool LDS = false>
__device__ __forceinline__ bool sm2_verify_lane26(const fe& hash_be, const uint8_t* sig, uint32_t siglen, CombTab tab,
                                                  fe& px, fe& py, uint32_t* ldsx = nullptr) {
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
    return sm2_verify_rs26<LDS>(hash_be, r, s, X, Y, tab, px, py, ldsx);
}

}  // namespace bcosgpu
