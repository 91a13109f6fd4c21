// ec_row.h -- Jacobian point arithmetic on row-spread field elements (fe_row.h) for the
// one-signature-per-workgroup kernels (ecc_row.hip): secp256k1 (FK1, a = 0) and SM2 (FSM2, a = -3).
//
// A point is REPLICATED over the wave's four DPP rows: every row holds X, Y and Z, each spread over
// its 16 lanes.  A formula runs as product LEVELS: in a level every row computes one product (its
// operands picked per row with v_cndmask), and gather4 (one v_permlane16_swap and two
// v_permlane32_swap) gives every row every row's product, so the point stays replicated.  A level
// costs one row product (~410 cycles, tools/rowbench.hip) plus ~10 instructions; a level with a
// single product needs no exchange at all (every row computes it).  The formulas are ec26.h's
// (dbl-2009-l with D = 4XB, madd-2007-bl with r carried as rr = r / 2) with the same magnitude schedule
// (fe_row.h keeps fe26.h's contracts):
//   dbl     : X, Y, Z <= 16 -> (10, 10, 2)                       3 levels
//   dbl_zz  : dbl + ZZ = Z3^2 (4), U2 = x ZZ, T = y Z3 (1)       3 levels
//   madd_zz : (10, 10, 2) after dbl_zz, (x, y) m <= 2 -> (9, 6, 2)    3 levels
// The mixed addition has no P = +-Q branches: it runs only inside the GLV chain, where (as the trio
// kernel's trio_add_digit argues) the accumulator K R with |K| >= 16 can never equal +-d R, |d| <= 8;
// infinity is the chain's own (wave-uniform) flag.
#pragma once
#include "fe26.h"
#include "fe_row.h"

namespace bcosgpu {
namespace frow {

struct Pt {
    uint32_t X, Y, Z;
};

// Field policies: the point formulas below are templates over the field's product, subtraction and
// negation (secp256k1: FK1; SM2: FSM2, with its own doubling for a = -3 and zero test further down).
struct FK1 {
    const Lane& L;
    __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const { return frow::mul(a, b, L); }
    template <int K>
    __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) const { return frow::sub<K>(a, b, L); }
    template <int K>
    __device__ __forceinline__ uint32_t neg(uint32_t a) const { return frow::neg<K>(a, L); }
};
struct FSM2 {
    const Lane& L;
    const Sm2Lane& C;
    __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const { return mul_sm2(a, b, L, C); }
    template <int K>
    __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) const { return sub_sm2<K>(a, b, C); }
    template <int K>
    __device__ __forceinline__ uint32_t neg(uint32_t a) const { return neg_sm2<K>(a, C); }
};

// L1 of a doubling: A = X^2 | B = Y^2 | W = Y Z (row 3 repeats row 2)
template <class F>
__device__ __forceinline__ Rows4 dbl_level1(const Pt& P, const F& f) {
    const Lane& L = f.L;
    return gather4(f.mul(sel4(L, P.X, P.Y, P.Y, P.Y), sel4(L, P.X, P.Y, P.Z, P.Z)));
}

// P = 2 P
template <class F>
__device__ __forceinline__ void dbl(Pt& P, const F& f) {
    const Lane& L = f.L;
    const Rows4 g1 = dbl_level1(P, f);
    const uint32_t B = g1.v[1], W = g1.v[2];
    const uint32_t E = mul_int<3>(g1.v[0]);  // 3 A                    m 3
    // L2: F = E^2 | C = B^2 | X B
    const Rows4 g2 = gather4(f.mul(sel4(L, E, B, P.X, P.X), sel4(L, E, B, B, B)));
    const uint32_t C = g2.v[1], D = mul_int<4>(g2.v[2]);  // D = 4 X B       m 4
    const uint32_t X3 = f.template sub<9>(g2.v[0], mul_int<2>(D));  // E^2 - 2 D   m 10
    const uint32_t t = f.template sub<11>(D, X3);                   // D - X3      m 15
    // L3: E (D - X3), one product: every row computes it
    const uint32_t Y3 = f.template sub<9>(f.mul(E, t), mul_int<8>(C));  // E (D - X3) - 8 C   m 10
    P.X = X3;
    P.Y = Y3;
    P.Z = mul_int<2>(W);  // 2 Y Z                                      m 2
}

// P = 2 P, and for the mixed addition of (x, y) that follows: ZZ = Z3^2, U2 = x ZZ, T = y Z3
template <class F>
__device__ __forceinline__ void dbl_zz(Pt& P, uint32_t x, uint32_t y, uint32_t& ZZ, uint32_t& U2, uint32_t& T,
                                       const F& f) {
    const Lane& L = f.L;
    const Rows4 g1 = dbl_level1(P, f);
    const uint32_t B = g1.v[1], W = g1.v[2];
    const uint32_t E = mul_int<3>(g1.v[0]);
    // L2: F = E^2 | C = B^2 | X B | W^2
    const Rows4 g2 = gather4(f.mul(sel4(L, E, B, P.X, W), sel4(L, E, B, B, W)));
    const uint32_t C = g2.v[1], D = mul_int<4>(g2.v[2]);
    const uint32_t X3 = f.template sub<9>(g2.v[0], mul_int<2>(D));
    const uint32_t t = f.template sub<11>(D, X3);
    const uint32_t Z3 = mul_int<2>(W);
    ZZ = mul_int<4>(g2.v[3]);  // (2 W)^2                              m 4
    // L3: E (D - X3) | x ZZ | y Z3
    const Rows4 g3 = gather4(f.mul(sel4(L, E, x, y, y), sel4(L, t, ZZ, Z3, Z3)));
    P.X = X3;
    P.Y = f.template sub<9>(g3.v[0], mul_int<8>(C));
    P.Z = Z3;
    U2 = g3.v[1];
    T = g3.v[2];
}

// P = P + (x, y) after dbl_zz (S2 = T ZZ = y Z^3)
template <class F>
__device__ __forceinline__ void madd_zz(Pt& P, uint32_t ZZ, uint32_t U2, uint32_t T, const F& f, uint32_t* Ho = nullptr,
                                        uint32_t* rro = nullptr) {
    const Lane& L = f.L;
    const uint32_t H = f.template sub<11>(U2, P.X);  // U2 - X1                    m 12
    // La: HH = H^2 | S2 = T ZZ | Z H
    const Rows4 ga = gather4(f.mul(sel4(L, H, T, P.Z, P.Z), sel4(L, H, ZZ, H, H)));
    const uint32_t I = mul_int<4>(ga.v[0]);        // 4 HH              m 4
    const uint32_t rr = f.template sub<11>(ga.v[1], P.Y);  // S2 - Y1 = r / 2   m 12
    // Lb: J = H I | V = X I | rr^2
    const Rows4 gb = gather4(f.mul(sel4(L, H, P.X, rr, rr), sel4(L, I, I, rr, rr)));
    const uint32_t J = gb.v[0], V = gb.v[1];
    uint32_t X3 = f.template sub<2>(mul_int<4>(gb.v[2]), J);  // r^2 - J         m 6
    X3 = f.template sub<3>(X3, mul_int<2>(V));                // - 2 V           m 9
    const uint32_t u = f.template sub<10>(V, X3);             // V - X3          m 11
    // Lc: rr (V - X3) | Y J
    uint32_t ya, yb;
    gather01(f.mul(sel4(L, rr, P.Y, P.Y, P.Y), sel4(L, u, J, J, J)), ya, yb);
    P.X = X3;
    P.Y = mul_int<2>(f.template sub<2>(ya, yb));  // r (V - X3) - 2 Y1 J       m 6
    P.Z = mul_int<2>(ga.v[2]);             // 2 Z1 H                   m 2
    if (Ho) *Ho = H;
    if (rro) *rro = rr;
}

// k (phi ? lambda : 1) P for the top 4 W bits of k held in SGPRs (k.v[0..3], wave-uniform; W = 32: a
// 128-bit k, W = 16: a 64-bit k in k.v[2..3] with k.v[0..1] = 0) over the co-Z table tab[8][3][16] (x, y,
// beta x of 1P .. 8P as row limbs of magnitude <= 1, lanes 10..15 zero): the trio kernel's radix-16
// Booth windows (the top digit = bit 127, then W windows of 4 doublings and one addition), neg
// negating every digit.  The digits, the infinity flag and every branch are wave-uniform.  Returns false
// when the result is infinity.
template <int W, class F>
__device__ __forceinline__ bool glv_chain(Pt& acc, fe& k, bool neg, bool phi, const uint32_t* tab, const F& f) {
    const Lane& L = f.L;
    const uint32_t one = L.one;
    bool inf = true;
    int d = static_cast<int>(k.v[3] >> 31);
    if (d != 0) {
        acc.X = tab[(phi ? 32 : 0) + L.k];
        acc.Y = tab[16 + L.k];
        if (neg) acc.Y = f.template neg<2>(acc.Y);
        acc.Z = one;
        inf = false;
    }
#pragma unroll 1
    for (int w = W - 1; w >= 0; --w) {
        d = booth_digit128(k);
        const int m = (d < 0 ? -d : d) - 1;
        const uint32_t* e = tab + (m & 7) * 48;
        const uint32_t x = e[(phi ? 32 : 0) + L.k];
        uint32_t y = e[16 + L.k];
        if ((d < 0) != neg) y = f.template neg<2>(y);
        if (inf) {
            if (d != 0) {
                acc.X = x;
                acc.Y = y;
                acc.Z = one;
                inf = false;
            }
            continue;
        }
        dbl(acc, f);
        dbl(acc, f);
        dbl(acc, f);
        if (d != 0) {
            uint32_t ZZ, U2, T;
            dbl_zz(acc, x, y, ZZ, U2, T, f);
            madd_zz(acc, ZZ, U2, T, f);
        } else {
            dbl(acc, f);
        }
    }
    return !inf;
}

// ------------------------------------------------------------------ levels, conversions, tables
// one product level with a product per row: every row receives all four
template <class F>
__device__ __forceinline__ Rows4 level(const F& f, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                                       uint32_t b2, uint32_t a3, uint32_t b3) {
    const Lane& L = f.L;
    return gather4(f.mul(sel4(L, a0, a1, a2, a3), sel4(L, b0, b1, b2, b3)));
}

// a fe26 held whole by every lane -> the row form (its limbs as they are)
__device__ __forceinline__ uint32_t from_fe26(const fe26& a, const Lane& L) {
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 10; ++q) w = L.k == q ? a.v[q] : w;
    return w;
}
// eight little-endian words (a canonical value, e.g. a comb entry in global memory) -> the row form
__device__ __forceinline__ uint32_t from_words(const uint32_t* w, const Lane& L) {
    const int bit = 26 * (L.k < 10 ? L.k : 0), i = bit >> 5, sh = bit & 31;
    const uint32_t lo = w[i], hi = i < 7 ? w[i + 1] : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, sh) & (M26 & L.lt10);
}
// ten row limbs (row magnitude <= 16: limbs < 2^31) -> fe26 of magnitude <= 2
__device__ __forceinline__ void fe26_from_row(fe26& r, const uint32_t* l) {
    using f26::M22;
    uint64_t t = 0;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        t += l[q];
        r.v[q] = static_cast<uint32_t>(t) & M26;
        t >>= 26;
    }
    // bits from 2^256 up: x 2^256 = x 977 + x 2^32 (mod p)
    const uint64_t x = (r.v[9] >> 22) + (t << 4);
    r.v[9] &= M22;
    uint64_t u = r.v[0] + x * 977u;
    r.v[0] = static_cast<uint32_t>(u) & M26;
    u = (u >> 26) + r.v[1] + (x << 6);
    r.v[1] = static_cast<uint32_t>(u) & M26;
#pragma unroll
    for (int q = 2; q < 9; ++q) {
        u = (u >> 26) + r.v[q];
        r.v[q] = static_cast<uint32_t>(u) & M26;
    }
    r.v[9] += static_cast<uint32_t>(u >> 26);
    F26_SETM(r, 2);
}
// a row element -> fe26 (magnitude <= 2) on every lane, through the wave's 16-word LDS slot
__device__ __forceinline__ void to_fe26(fe26& r, uint32_t x, uint32_t* slot, const Lane& L) {
    if (L.row == 0) slot[L.k] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t l[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) l[q] = slot[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    fe26_from_row(r, l);
}
// x == 0 (mod p), as a wave-uniform (SGPR) flag: every branch on it is a scalar branch
__device__ __forceinline__ bool is_zero(uint32_t x, uint32_t* slot, const Lane& L) {
    fe26 t;
    to_fe26(t, x, slot, L);
    return __builtin_amdgcn_readfirstlane(fe26_is_zero(t) ? 1u : 0u) != 0u;
}

// R = P + Q in Jacobian coordinates, P != +-Q, neither at infinity (add-2007-bl as ec26.h's
// CurveK1x::add): P, Q m <= 16 -> (6, 4, 2), 5 levels; H = U2 - U1 and rr = 2 (S2 - S1) returned for
// the complete addition's tests
template <class F>
__device__ __forceinline__ void add_inc(Pt& R, const Pt& P, const Pt& Q, const F& f, uint32_t* Ho = nullptr,
                                        uint32_t* rro = nullptr) {
    const Lane& L = f.L;
    const Rows4 g1 = level(f, P.Z, P.Z, Q.Z, Q.Z, P.Y, Q.Z, Q.Y, P.Z);  // Z1Z1 | Z2Z2 | Y1 Z2 | Y2 Z1
    const Rows4 g2 = level(f, P.X, g1.v[1], Q.X, g1.v[0], g1.v[2], g1.v[1], g1.v[3], g1.v[0]);  // U1 | U2 | S1 | S2
    const uint32_t U1 = g2.v[0], S1 = g2.v[2];
    const uint32_t H = f.template sub<2>(g2.v[1], U1);              // U2 - U1          m 3
    const uint32_t t = mul_int<2>(H);                       // 2 H              m 6
    const uint32_t rr = mul_int<2>(f.template sub<2>(g2.v[3], S1));  // 2 (S2 - S1)      m 6
    const Rows4 g3 = level(f, t, t, rr, rr, P.Z, Q.Z, P.Z, Q.Z);  // I = (2H)^2 | rr^2 | Z1 Z2
    const uint32_t I = g3.v[0];
    const Rows4 g4 = level(f, H, I, U1, I, g3.v[2], H, g3.v[2], H);  // J = H I | V = U1 I | Z1 Z2 H
    const uint32_t J = g4.v[0], V = g4.v[1];
    uint32_t X3 = f.template sub<2>(g3.v[1], J);  // rr^2 - J                             m 3
    X3 = f.template sub<3>(X3, mul_int<2>(V));    // - 2 V                                m 6
    const uint32_t u = f.template sub<7>(V, X3);  // V - X3                               m 8
    uint32_t ya, yb;
    gather01(f.mul(sel4(L, rr, S1, S1, S1), sel4(L, u, J, J, J)), ya, yb);
    R.X = X3;
    R.Y = f.template sub<3>(ya, mul_int<2>(yb));  // rr (V - X3) - 2 S1 J                m 4
    R.Z = mul_int<2>(g4.v[2]);            // 2 Z1 Z2 H                           m 2
    if (Ho) *Ho = H;
    if (rro) *rro = rr;
}

// R = P + Q, complete: infinity on either side, P = Q (doubling), P = -Q (infinity) -- ec26.h's cases.
// Every flag and test is wave-uniform.
template <class F>
__device__ __forceinline__ void add_full(Pt& R, bool& rinf, const Pt& P, bool pinf, const Pt& Q, bool qinf,
                                         uint32_t* slot, const F& f) {
    if (pinf) {
        R = Q;
        rinf = qinf;
        return;
    }
    if (qinf) {
        R = P;
        rinf = false;
        return;
    }
    Pt S;
    uint32_t H, rr;
    add_inc(S, P, Q, f, &H, &rr);
    rinf = false;
    if (field_is_zero(H, slot, f)) {
        if (field_is_zero(rr, slot, f)) {
            S = P;
            curve_dbl(S, f);
        } else {
            rinf = true;
        }
    }
    R = S;
}

// P = P + (x, y), (x, y) affine m <= 2, P != +-(x, y), P not at infinity: 5 levels -> (9, 6, 2)
template <class F>
__device__ __forceinline__ void madd(Pt& P, uint32_t x, uint32_t y, const F& f) {
    const Lane& L = f.L;
    uint32_t ZZ, T;
    gather01(f.mul(sel4(L, P.Z, y, y, y), sel4(L, P.Z, P.Z, P.Z, P.Z)), ZZ, T);  // Z^2 | y Z
    const uint32_t U2 = f.mul(x, ZZ);                                           // (every row)
    madd_zz(P, ZZ, U2, T, f);
}

// The GLV table of a point P1 (Jacobian, magnitudes <= 16, of order n): 1P .. 8P rescaled to the common
// Zc = Z1 ... Z8 (entries affine on the curve y^2 = x^3 + 7 Zc^6 w^3, as coz_table26) -> tab[j][0] = x,
// tab[j][1] = y, tab[j][2] = beta x (row limbs, magnitude 1), zc = Zc.  The additions never meet
// P = +-Q (jP +- P for j <= 6 and P of order n); an invalid P only yields a table whose verdict is
// already false.
template <class F, bool BETA = true>
__device__ __forceinline__ void build_table(uint32_t (*tab)[3][16], uint32_t* zc, const Pt& P1, uint32_t beta,
                                            const F& f) {
    const Lane& L = f.L;
    Pt T[8];
    T[0] = P1;
    T[1] = P1;
    curve_dbl(T[1], f);
    add_inc(T[2], T[1], T[0], f);
    T[3] = T[1];
    curve_dbl(T[3], f);
    add_inc(T[4], T[3], T[0], f);
    T[5] = T[2];
    curve_dbl(T[5], f);
    add_inc(T[6], T[5], T[0], f);
    T[7] = T[3];
    curve_dbl(T[7], f);
    // prefix and suffix products of the Z's, side by side (rows 0 / 1)
    uint32_t pre[8], suf[8];
    pre[0] = T[0].Z;
    suf[7] = T[7].Z;
#pragma unroll
    for (int j = 1; j < 8; ++j)
        gather01(f.mul(sel4(L, pre[j - 1], suf[8 - j], suf[8 - j], suf[8 - j]),
                     sel4(L, T[j].Z, T[7 - j].Z, T[7 - j].Z, T[7 - j].Z)),
                 pre[j], suf[7 - j]);
    // s_j = Zc / Z_j = pre_(j-1) suf_(j+1)
    uint32_t sj[8], s2[8], s3[8], xs[8];
    sj[0] = suf[1];
    sj[7] = pre[6];
    {
        const Rows4 g = level(f, pre[0], suf[2], pre[1], suf[3], pre[2], suf[4], pre[3], suf[5]);
        sj[1] = g.v[0];
        sj[2] = g.v[1];
        sj[3] = g.v[2];
        sj[4] = g.v[3];
        uint32_t a, b;
        gather01(f.mul(sel4(L, pre[4], pre[5], pre[5], pre[5]), sel4(L, suf[6], suf[7], suf[7], suf[7])), a, b);
        sj[5] = a;
        sj[6] = b;
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
        const Rows4 g = level(f, sj[j], sj[j], sj[j + 1], sj[j + 1], sj[j + 2], sj[j + 2], sj[j + 3], sj[j + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) s2[j + q] = g.v[q];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {  // s^3 and X s^2 of two entries per level
        const Rows4 g = level(f, s2[j], sj[j], T[j].X, s2[j], s2[j + 1], sj[j + 1], T[j + 1].X, s2[j + 1]);
        s3[j] = g.v[0];
        xs[j] = g.v[1];
        s3[j + 1] = g.v[2];
        xs[j + 1] = g.v[3];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {  // Y s^3
        const Rows4 g = level(f, T[j].Y, s3[j], T[j + 1].Y, s3[j + 1], T[j + 2].Y, s3[j + 2], T[j + 3].Y, s3[j + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (L.row == 0 && L.k < 16) tab[j + q][1][L.k] = g.v[q];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {  // beta x
        Rows4 g{{0u, 0u, 0u, 0u}};
        if constexpr (BETA) g = level(f, beta, xs[j], beta, xs[j + 1], beta, xs[j + 2], beta, xs[j + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (L.row == 0) {
                tab[j + q][0][L.k] = xs[j + q];
                tab[j + q][2][L.k] = g.v[q];
            }
    }
    if (L.row == 0) zc[L.k] = pre[7];
}

// a^((p+1)/4): a square root of a when one exists (fe26_sqrt_cand's chain on the rows; a m <= 2)
template <class F>
__device__ __forceinline__ uint32_t sqr_n(uint32_t a, int n, const F& f) {
    uint32_t t = f.mul(a, a);
#pragma unroll 1
    for (int i = 1; i < n; ++i) t = f.mul(t, t);
    return t;
}
template <class F>
__device__ __forceinline__ uint32_t sqrt_cand(uint32_t a, const F& f) {
    const uint32_t x2 = f.mul(f.mul(a, a), a);
    const uint32_t x3 = f.mul(f.mul(x2, x2), a);
    const uint32_t x6 = f.mul(sqr_n(x3, 3, f), x3);
    const uint32_t x9 = f.mul(sqr_n(x6, 3, f), x3);
    const uint32_t x11 = f.mul(sqr_n(x9, 2, f), x2);
    const uint32_t x22 = f.mul(sqr_n(x11, 11, f), x11);
    const uint32_t x44 = f.mul(sqr_n(x22, 22, f), x22);
    const uint32_t x88 = f.mul(sqr_n(x44, 44, f), x44);
    const uint32_t x176 = f.mul(sqr_n(x88, 88, f), x88);
    const uint32_t x220 = f.mul(sqr_n(x176, 44, f), x44);
    const uint32_t x223 = f.mul(sqr_n(x220, 3, f), x3);
    uint32_t t = f.mul(sqr_n(x223, 23, f), x22);
    t = f.mul(sqr_n(t, 6, f), x2);
    return sqr_n(t, 2, f);
}

// ------------------------------------------------------------------ SM2 (a = -3)
// doubling dbl-2001-b: delta = Z^2, gamma = Y^2, beta = X gamma, alpha = 3 (X - delta)(X + delta),
// X3 = alpha^2 - 8 beta, Z3 = 2 Y Z, Y3 = alpha (4 beta - X3) - 8 gamma^2: 4 levels, X <= 12, Y, Z <= 16
// -> (10, 10, 2)
template <class F>
__device__ __forceinline__ void dbl_m3(Pt& P, const F& f) {
    const Lane& L = f.L;
    const Rows4 g1 = gather4(f.mul(sel4(L, P.Z, P.Y, P.Y, P.Y), sel4(L, P.Z, P.Y, P.Z, P.Z)));  // delta | gamma | Y Z
    const uint32_t dl = g1.v[0], gm = g1.v[1], W = g1.v[2];
    const uint32_t xm = f.template sub<2>(P.X, dl), xp = P.X + dl;  // m X + 2, X + 1
    const Rows4 g2 = gather4(f.mul(sel4(L, P.X, xm, gm, gm), sel4(L, gm, xp, gm, gm)));  // beta | (X-d)(X+d) | gamma^2
    const uint32_t b4 = mul_int<4>(g2.v[0]), al = mul_int<3>(g2.v[1]), C = g2.v[2];
    const uint32_t X3 = f.template sub<9>(f.mul(al, al), mul_int<2>(b4));  // alpha^2 - 8 beta     m 10
    const uint32_t t = f.template sub<11>(b4, X3);                           // 4 beta - X3          m 15
    P.Y = f.template sub<9>(f.mul(al, t), mul_int<8>(C));                     // m 10
    P.X = X3;
    P.Z = mul_int<2>(W);
}
// the chain's doubling with ZZ = Z^2 carried beside the point (m <= 16), so that alpha = 3 (X^2 - ZZ^2)
// is ready after the first level: 3 levels -- X^2 | gamma = Y^2 | Y Z | ZZ^2, then alpha^2 | beta = X gamma |
// gamma^2 | gamma ZZ (Z3^2 = 4 gamma ZZ), then alpha (4 beta - X3) -- and (10, 10, 2), ZZ 4
template <class F>
__device__ __forceinline__ void dbl_m3z(Pt& P, uint32_t& ZZ, const F& f) {
    const Lane& L = f.L;
    const Rows4 g1 = gather4(f.mul(sel4(L, P.X, P.Y, P.Y, ZZ), sel4(L, P.X, P.Y, P.Z, ZZ)));
    const uint32_t gm = g1.v[1], W = g1.v[2];
    const uint32_t al = mul_int<3>(f.template sub<2>(g1.v[0], g1.v[3]));  // 3 (X^2 - Z^4)       m 9
    const Rows4 g2 = gather4(f.mul(sel4(L, al, P.X, gm, gm), sel4(L, al, gm, gm, ZZ)));
    const uint32_t b4 = mul_int<4>(g2.v[1]), C = g2.v[2];
    const uint32_t X3 = f.template sub<9>(g2.v[0], mul_int<2>(b4));  // alpha^2 - 8 beta    m 10
    const uint32_t t = f.template sub<11>(b4, X3);                   // 4 beta - X3         m 15
    P.Y = f.template sub<9>(f.mul(al, t), mul_int<8>(C));             // m 10
    P.X = X3;
    P.Z = mul_int<2>(W);
    ZZ = mul_int<4>(g2.v[3]);
}
// the window's last doubling (dbl_m3z) with, beside alpha (4 beta - X3) in level 3, the addition's
// U2 = x Z3^2, T = y Z3 and U1 = X3 Zc^2 (the table entry (x, y) is the Jacobian point (x, y, Zc))
template <class F>
__device__ __forceinline__ void dbl_m3z_zz(Pt& P, uint32_t& ZZ, uint32_t x, uint32_t y, uint32_t zc2, uint32_t& U2,
                                           uint32_t& T, uint32_t& U1, const F& f) {
    const Lane& L = f.L;
    const Rows4 g1 = gather4(f.mul(sel4(L, P.X, P.Y, P.Y, ZZ), sel4(L, P.X, P.Y, P.Z, ZZ)));
    const uint32_t gm = g1.v[1];
    const uint32_t al = mul_int<3>(f.template sub<2>(g1.v[0], g1.v[3]));
    const uint32_t Z3 = mul_int<2>(g1.v[2]);
    const Rows4 g2 = gather4(f.mul(sel4(L, al, P.X, gm, gm), sel4(L, al, gm, gm, ZZ)));
    const uint32_t b4 = mul_int<4>(g2.v[1]), C = g2.v[2];
    const uint32_t X3 = f.template sub<9>(g2.v[0], mul_int<2>(b4));
    const uint32_t t = f.template sub<11>(b4, X3);
    ZZ = mul_int<4>(g2.v[3]);
    const Rows4 g3 = gather4(f.mul(sel4(L, al, x, y, X3), sel4(L, t, ZZ, Z3, zc2)));  // alpha t | U2 | T | U1
    P.Y = f.template sub<9>(g3.v[0], mul_int<8>(C));
    P.X = X3;
    P.Z = Z3;
    U2 = g3.v[1];
    T = g3.v[2];
    U1 = g3.v[3];
}

// P = P + (x, y, Zc) after dbl_m3z_zz: the table entry is a Jacobian point with the table's common Z = Zc
// (SM2's doubling needs true coordinates: on the co-Z rescaled curve a would become -3 Zc^4), so
// U1 = X1 Zc^2 (from the doubling), S1 = Y1 Zc^3, Z3 = 2 Z1 Zc H and the next ZZ = Z3^2 join the spare rows
// of madd_zz's three levels.  P (10, 10, 2), (x, y) m <= 2 -> (9, 6, 2), ZZ 4; H and rr = S2 - S1 returned
// for the complete last addition
template <class F>
__device__ __forceinline__ void add_coz_zz(Pt& P, uint32_t& ZZ, uint32_t U2, uint32_t T, uint32_t U1, uint32_t zc,
                                           uint32_t zc3, const F& f, uint32_t* Ho = nullptr, uint32_t* rro = nullptr) {
    const Lane& L = f.L;
    const uint32_t H = f.template sub<2>(U2, U1);  // m 3
    // La: HH | S1 = Y1 Zc^3 | S2 = T ZZ | Z1 H
    const Rows4 ga = gather4(f.mul(sel4(L, H, P.Y, T, P.Z), sel4(L, H, zc3, ZZ, H)));
    const uint32_t I = mul_int<4>(ga.v[0]), S1 = ga.v[1];
    const uint32_t rr = f.template sub<2>(ga.v[2], S1);  // S2 - S1 = r / 2          m 3
    // Lb: J = H I | V = U1 I | rr^2 | Z1 H Zc
    const Rows4 gb = gather4(f.mul(sel4(L, H, U1, rr, ga.v[3]), sel4(L, I, I, rr, zc)));
    const uint32_t J = gb.v[0], V = gb.v[1];
    uint32_t X3 = f.template sub<2>(mul_int<4>(gb.v[2]), J);  // r^2 - J                m 6
    X3 = f.template sub<3>(X3, mul_int<2>(V));                // - 2 V                  m 9
    const uint32_t u = f.template sub<10>(V, X3);             // V - X3                 m 11
    // Lc: rr (V - X3) | S1 J | (Z1 H Zc)^2
    const uint32_t zh = gb.v[3];
    const Rows4 gc = gather4(f.mul(sel4(L, rr, S1, zh, zh), sel4(L, u, J, zh, zh)));
    P.X = X3;
    P.Y = mul_int<2>(f.template sub<2>(gc.v[0], gc.v[1]));  // r (V - X3) - 2 S1 J   m 6
    P.Z = mul_int<2>(zh);                                    // 2 Z1 Zc H            m 2
    ZZ = mul_int<4>(gc.v[2]);                                // Z3^2                 m 4
    if (Ho) *Ho = H;
    if (rro) *rro = rr;
}

// x == 0 (mod p_SM2), wave-uniform: the value (< 2^265) as nine words, the bits from 2^256 folded once by
// 2^256 = 2^224 + 2^96 - 2^64 + 1 (mod p), which leaves it below 2p: zero iff it is 0 or p
__device__ __forceinline__ bool is_zero_sm2(uint32_t x, uint32_t* slot, const Lane& L) {
    if (L.row == 0) slot[L.k] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t l[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) l[q] = slot[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t nl[10];  // carried into 26-bit limbs; the carry out of limb 9 is bit 260 and up
    uint32_t top = 0;
    {
        uint64_t t = 0;
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            t += l[q];
            nl[q] = static_cast<uint32_t>(t) & M26;
            t >>= 26;
        }
        top = static_cast<uint32_t>(t);
    }
    uint32_t w[9];
    w[0] = nl[0] | (nl[1] << 26);
    w[1] = (nl[1] >> 6) | (nl[2] << 20);
    w[2] = (nl[2] >> 12) | (nl[3] << 14);
    w[3] = (nl[3] >> 18) | (nl[4] << 8);
    w[4] = (nl[4] >> 24) | (nl[5] << 2) | (nl[6] << 28);
    w[5] = (nl[6] >> 4) | (nl[7] << 22);
    w[6] = (nl[7] >> 10) | (nl[8] << 16);
    w[7] = (nl[8] >> 16) | (nl[9] << 10);
    w[8] = (nl[9] >> 22) | (top << 4);
    const int64_t h = w[8];
    int64_t c = 0;
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        c += static_cast<int64_t>(w[i]) + (i == 0 ? h : 0) - (i == 2 ? h : 0) + (i == 3 ? h : 0) + (i == 7 ? h : 0);
        o[i] = static_cast<uint32_t>(c);
        c >>= 32;
    }
    constexpr uint32_t P2[8] = {0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu,
                                0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu};
    uint32_t z = 0, zp = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        z |= o[i];
        zp |= o[i] ^ P2[i];
    }
    const bool zero = c == 0 && (z == 0u || zp == 0u);
    return __builtin_amdgcn_readfirstlane(zero ? 1u : 0u) != 0u;
}

// t P for a 256-bit t held in SGPRs over the co-Z table tab[8][3][16] (x, y of 1P .. 8P, each the Jacobian
// point (x, y, Zc): the result is in true coordinates on E): radix-16 Booth
// windows (the top digit = bit 255, then 64 windows of 4 doublings and one addition, 15 levels).  Before every
// window but the last the accumulator is K P with 16 <= K < n / 16 + 8, which can never meet +-d P
// (|d| <= 8); at the last window K = t - d may (t = n - 2 |d| gives K = -d), so its addition is
// complete (zero tests on H and r, the doubling or infinity).  Returns false when the result is infinity.
template <class F>
__device__ __forceinline__ bool sm2_chain(Pt& acc, fe& k, const uint32_t* tab, uint32_t zc, uint32_t* slot,
                                          const F& f) {
    const Lane& L = f.L;
    const uint32_t zc2 = f.mul(zc, zc), zc3 = f.mul(zc2, zc);
    bool inf = true;
    uint32_t ZZ = zc2;
    int d = static_cast<int>(k.v[7] >> 31);
    if (d != 0) {
        acc.X = tab[L.k];
        acc.Y = tab[16 + L.k];
        acc.Z = zc;
        inf = false;
    }
#pragma unroll 1
    for (int w = 63; w >= 0; --w) {
        const uint32_t top = k.v[7];
        const uint32_t Wd = top >> 28, c = (top >> 27) & 1u;
        d = static_cast<int>(Wd + c) - static_cast<int>((Wd >> 3) << 4);
        shl4(k);
        const int m = (d < 0 ? -d : d) - 1;
        const uint32_t* e = tab + (m & 7) * 48;
        const uint32_t x = e[L.k];
        uint32_t y = e[16 + L.k];
        if (d < 0) y = f.template neg<2>(y);
        if (inf) {
            if (d != 0) {
                acc.X = x;
                acc.Y = y;
                acc.Z = zc;
                ZZ = zc2;
                inf = false;
            }
            continue;
        }
        dbl_m3z(acc, ZZ, f);
        dbl_m3z(acc, ZZ, f);
        dbl_m3z(acc, ZZ, f);
        if (d != 0) {
            uint32_t U2, T, U1, H, rr;
            dbl_m3z_zz(acc, ZZ, x, y, zc2, U2, T, U1, f);
            if (w != 0) {
                add_coz_zz(acc, ZZ, U2, T, U1, zc, zc3, f);
            } else {
                const Pt before = acc;
                const uint32_t zzb = ZZ;
                add_coz_zz(acc, ZZ, U2, T, U1, zc, zc3, f, &H, &rr);
                if (is_zero_sm2(H, slot, L)) {
                    if (is_zero_sm2(rr, slot, L)) {
                        acc = before;
                        ZZ = zzb;
                        dbl_m3z(acc, ZZ, f);
                    } else {
                        inf = true;
                    }
                }
            }
        } else {
            dbl_m3z(acc, ZZ, f);
        }
    }
    return !inf;
}

// the curve's doubling and the field's zero test for the generic formulas above
__device__ __forceinline__ void curve_dbl(Pt& P, const FK1& f) { dbl(P, f); }
__device__ __forceinline__ void curve_dbl(Pt& P, const FSM2& f) { dbl_m3(P, f); }
__device__ __forceinline__ bool field_is_zero(uint32_t x, uint32_t* slot, const FK1& f) { return is_zero(x, slot, f.L); }
__device__ __forceinline__ bool field_is_zero(uint32_t x, uint32_t* slot, const FSM2& f) {
    return is_zero_sm2(x, slot, f.L);
}

// a row point through LDS (48 words: X, Y, Z), written by row 0
__device__ __forceinline__ void pt_store(uint32_t (*d)[16], const Pt& P, const Lane& L) {
    if (L.row == 0) {
        d[0][L.k] = P.X;
        d[1][L.k] = P.Y;
        d[2][L.k] = P.Z;
    }
}
__device__ __forceinline__ void pt_load(Pt& P, const uint32_t (*d)[16], const Lane& L) {
    P.X = d[0][L.k];
    P.Y = d[1][L.k];
    P.Z = d[2][L.k];
}

}  // namespace frow
}  // namespace bcosgpu
