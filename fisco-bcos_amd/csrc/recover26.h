// recover26.h -- secp256k1 public-key recovery with the point arithmetic over the 10 x 26-bit field
// (fe26.h / ec26.h), for the throughput kernels (tx_verify_kernel<secp, *> and the recover / verify
// kernels).  Same algorithm, same decisions and same outputs as secp256k1_recover_rsv in
// ecc_device.h (libsecp256k1 secp256k1_ecdsa_recover semantics, as wedpr calls it from
// Secp256k1Crypto.cpp:79-93): the scalar work (range checks, r^-1 mod n, u1, u2, the GLV split) stays
// in the 8 x 32-bit code, the curve work -- sqrt, the GLV double-and-add over the co-Z table, the comb,
// the final addition -- runs on fe26, and the result is converted back to canonical words once.
// Included by ecc_device.h after its FieldK1 helpers (constants, glv_split, booth digits, CombTab).
#pragma once
#include "ec26.h"

namespace bcosgpu {

__device__ __forceinline__ void fe26_from_fe(fe26& r, const fe& a) { fe26_from_words(r, a.v); }
// canonical words
__device__ __forceinline__ void fe26_to_fe(fe& r, const fe26& a) {
    fe26 t;
    fe26_copy(t, a);
    fe26_normalize(t);
    fe26_to_words(r.v, t);
}
__device__ __forceinline__ void fe26_const(fe26& r, const uint32_t* k) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = k[i];
    fe26_from_words(r, w);
}

// one comb entry (x[8] || y[8], canonical words) -> affine fe26
__device__ __forceinline__ void load_aff26(Aff26& T, const uint32_t* __restrict__ e32) {
    const uint4* e = reinterpret_cast<const uint4*>(e32);
    const uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
    const uint32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const uint32_t y[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    fe26_from_words(T.x, x);
    fe26_from_words(T.y, y);
}

// acc = k * G over a BITS-bit comb table, as comb_mul: the next window's entry is fetched (as raw
// words) before the current addition
template <int BITS>
__device__ __forceinline__ void comb_mul26(Jac26& acc, const fe& k_plain, const uint32_t* __restrict__ tab) {
    constexpr int W = 256 / BITS;
    constexpr uint32_t E = 1u << BITS, MASK = E - 1u;
    fe k;
    fe_copy(k, k_plain);
    CurveK1x::set_inf(acc);
    uint32_t b = k.v[0] & MASK;
    shr_bits<BITS>(k);
    const uint4* e = reinterpret_cast<const uint4*>(tab + static_cast<size_t>(b) * 16);
    uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
#pragma unroll 1
    for (int i = 0; i < W; ++i) {
        const uint32_t bi = b;
        Aff26 T;
        {
            const uint32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
            const uint32_t y[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            fe26_from_words(T.x, x);
            fe26_from_words(T.y, y);
        }
        const int in = i + 1 < W ? i + 1 : i;  // last window: a harmless reload
        b = k.v[0] & MASK;
        shr_bits<BITS>(k);
        e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(in) * E + b) * 16);
        q0 = e[0];
        q1 = e[1];
        q2 = e[2];
        q3 = e[3];
        Jac26 S;
        CurveK1x::madd(S, acc, T);
        CurveK1x::cmov(acc, S, bi != 0u);
    }
}
__device__ __forceinline__ void comb_mul26_rt(Jac26& acc, const fe& k, CombTab tab) {
    if (tab.bits == kWideBits) comb_mul26<kWideBits>(acc, k, tab.p);
    else comb_mul26<8>(acc, k, tab.p);
}

// T[j] = (j + 1) P
__device__ __forceinline__ void multiples8_26(Jac26 T[8], const Aff26& P) {
    CurveK1x::from_aff(T[0], P);
    CurveK1x::dbl(T[1], T[0]);
    CurveK1x::madd(T[2], T[1], P);
    CurveK1x::dbl(T[3], T[1]);
    CurveK1x::madd(T[4], T[3], P);
    CurveK1x::dbl(T[5], T[2]);
    CurveK1x::madd(T[6], T[5], P);
    CurveK1x::dbl(T[7], T[3]);
}

// co-Z rescale of T[0..7] (T[0].Z == 1) to Zc = Z1 ... Z7, as coz_table_k1: the entries are affine on
// the isomorphic curve y^2 = x^3 + 7 Zc^6 (a = 0 kept), results are (X, Y, Z Zc) on the real curve
__device__ __forceinline__ void coz_table26(Aff26 A[8], fe26& Zc, const Jac26 T[8]) {
    // s_j = Zc / Z_j = (Z_1 ... Z_(j-1)) (Z_(j+1) ... Z_7): prefix products kept, the suffix as a running
    // product while the entries are emitted from the top down (T[7] is released first)
    fe26 pre[7], suf;
    fe26_one(pre[0]);
    fe26_copy(pre[1], T[1].Z);
    Unroll<2, 7>::run([&](auto J) { fe26_mul(pre[J], pre[J - 1], T[J].Z); });
    fe26_mul(Zc, pre[6], T[7].Z);
    Unroll<0, 8>::run([&](auto J) {
        constexpr int j = 7 - decltype(J)::value;
        fe26 sj, s2, s3;
        if constexpr (j == 7) fe26_copy(sj, pre[6]);
        else if constexpr (j <= 1) fe26_copy(sj, suf);
        else fe26_mul(sj, pre[j - 1], suf);
        if constexpr (j == 7) fe26_copy(suf, T[7].Z);
        else if constexpr (j >= 1) fe26_mul(suf, suf, T[j].Z);
        fe26_sqr(s2, sj);
        fe26_mul(s3, s2, sj);
        fe26_mul(A[j].x, T[j].X, s2);
        fe26_mul(A[j].y, T[j].Y, s3);
    });
}

// acc += (sign d) (phi ? lambda : 1) P from the table: x-coordinates as canonical words in the wave's
// LDS slice ([entry][word][lane], ldsx offset by the lane), y-coordinates as canonical words in
// registers (8 per entry instead of 10: the window loop of the occupancy-2 kernel is register-bound)
__device__ __forceinline__ void add_digit26(Jac26& acc, const uint32_t* ldsx, const fe Y[8], const fe26& beta,
                                            int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    Aff26 S;
    {
        const uint32_t* b = ldsx + m * 512u;
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = b[k * 64];
        fe26_from_words(S.x, w);
    }
    {
        fe y;
        fe_copy(y, Y[0]);
#pragma unroll
        for (int q = 1; q < 8; ++q) fe_cmov(y, Y[q], m == static_cast<uint32_t>(q));
        fe26_from_fe(S.y, y);
    }
    if (phi) fe26_mul(S.x, S.x, beta);
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    Jac26 R;
    CurveK1x::madd(R, acc, S);
    CurveK1x::cmov(acc, R, d != 0);
}

// acc += ... from a register table (LDS = false variant)
__device__ __forceinline__ void add_digit26_reg(Jac26& acc, const Aff26 A[8], const fe26& beta, int d, bool neg,
                                                bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    Aff26 S;
    fe26_copy(S.x, A[0].x);
    fe26_copy(S.y, A[0].y);
#pragma unroll
    for (int q = 1; q < 8; ++q) {
        const bool take = m == static_cast<uint32_t>(q);
        fe26_cmov(S.x, A[q].x, take);
        fe26_cmov(S.y, A[q].y, take);
    }
    if (phi) fe26_mul(S.x, S.x, beta);
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    Jac26 R;
    CurveK1x::madd(R, acc, S);
    CurveK1x::cmov(acc, R, d != 0);
}

// acc = k P via GLV, 33 joint radix-16 Booth windows against the co-Z table (glv_mul_k1)
template <bool LDS>
__device__ __forceinline__ void glv_mul_k1_26(Jac26& acc, const fe& k, const Aff26& P, uint32_t* ldsx) {
    fe k1, k2;
    bool neg1, neg2;
    glv_split(k1, neg1, k2, neg2, k);
    Aff26 A[8];
    fe26 Zc, beta;
    {
        Jac26 T[8];
        multiples8_26(T, P);
        coz_table26(A, Zc, T);
    }
    fe26_const(beta, kGlvBeta);
    CurveK1x::set_inf(acc);
    if constexpr (LDS) {
        fe Y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            fe x;
            fe26_to_fe(x, A[j].x);
#pragma unroll
            for (int w = 0; w < 8; ++w) ldsx[(j * 8 + w) * 64] = x.v[w];
            fe26_to_fe(Y[j], A[j].y);
        }
        add_digit26(acc, ldsx, Y, beta, static_cast<int>(k1.v[3] >> 31), neg1, false);
        add_digit26(acc, ldsx, Y, beta, static_cast<int>(k2.v[3] >> 31), neg2, true);
#pragma unroll 1
        for (int i = 31; i >= 0; --i) {
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            const int d1 = booth_digit128(k1);
            const int d2 = booth_digit128(k2);
            add_digit26(acc, ldsx, Y, beta, d1, neg1, false);
            add_digit26(acc, ldsx, Y, beta, d2, neg2, true);
        }
    } else {
        add_digit26_reg(acc, A, beta, static_cast<int>(k1.v[3] >> 31), neg1, false);
        add_digit26_reg(acc, A, beta, static_cast<int>(k2.v[3] >> 31), neg2, true);
#pragma unroll 1
        for (int i = 31; i >= 0; --i) {
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            CurveK1x::dbl(acc, acc);
            const int d1 = booth_digit128(k1);
            const int d2 = booth_digit128(k2);
            add_digit26_reg(acc, A, beta, d1, neg1, false);
            add_digit26_reg(acc, A, beta, d2, neg2, true);
        }
    }
    fe26_mul(acc.Z, acc.Z, Zc);
}

// secp256k1_recover_rsv on fe26 (same contract)
template <bool LDS = false>
__device__ __forceinline__ bool secp256k1_recover_rsv26(const fe& hash_be, const fe& r, const fe& s, uint32_t v,
                                                        CombTab tab, fe& px, fe& py, uint32_t* ldsx = nullptr) {
    bool ok = v <= 3u;
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, ParamN1::M);
    fe x;
    fe_copy(x, r);
    if (v & 2u) {
        ok = ok && fe_lt_k(r, kK1PminusN);
        fe_add_k(x, r, ParamN1::M);
    }
    // y = sqrt(x^3 + 7), y parity = v & 1
    fe26 X, rhs, y, t, seven;
    fe26_from_fe(X, x);
    fe26_sqr(t, X);
    fe26_mul(rhs, t, X);
    fe26_set_small(seven, 7u);
    fe26_add(rhs, rhs, seven);
    fe26_sqrt_cand(y, rhs);
    fe26_sqr(t, y);
    fe26_sub<3>(t, t, rhs);
    ok = ok && fe26_is_zero(t);
    fe26_normalize(y);
    fe26 ny;
    fe26_neg<2>(ny, y);
    fe26_normalize(ny);
    fe26_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
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
    // Q = u1 G + u2 R
    Aff26 R;
    fe26_copy(R.x, X);
    fe26_copy(R.y, y);
    Jac26 QG, QR, Q;
    glv_mul_k1_26<LDS>(QR, u2, R, ldsx);
    comb_mul26_rt(QG, u1, tab);
    CurveK1x::add(Q, QG, QR);
    ok = ok && !Q.inf;
    // affine: one inversion of Z on the 8 x 32-bit side
    fe z, zi;
    fe26_to_fe(z, Q.Z);
    FieldInv<FieldK1>::inv(zi, z);
    fe26 zi26, zi2, zi3, ax, ay;
    fe26_from_fe(zi26, zi);
    fe26_sqr(zi2, zi26);
    fe26_mul(ax, Q.X, zi2);
    fe26_mul(zi3, zi2, zi26);
    fe26_mul(ay, Q.Y, zi3);
    fe26_to_fe(px, ax);
    fe26_to_fe(py, ay);
    return ok;
}

template <bool LDS = false>
__device__ __forceinline__ bool secp256k1_recover_lane26(const fe& hash_be, const uint8_t* sig, uint32_t siglen,
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
    return secp256k1_recover_rsv26<LDS>(hash_be, r, s, rd.word(16) & 0xffu, tab, px, py, ldsx);
}

}  // namespace bcosgpu
