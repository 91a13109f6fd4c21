// ec_row.h -- secp256k1 Jacobian point arithmetic on row-spread field elements (fe_row.h), for the
// one-signature-per-workgroup recovery kernel (ecc_row.hip).
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

// L1 of a doubling: A = X^2 | B = Y^2 | W = Y Z (row 3 repeats row 2)
__device__ __forceinline__ Rows4 dbl_level1(const Pt& P, const Lane& L) {
    return gather4(mul(sel4(L, P.X, P.Y, P.Y, P.Y), sel4(L, P.X, P.Y, P.Z, P.Z), L));
}

// P = 2 P
__device__ __forceinline__ void dbl(Pt& P, const Lane& L) {
    const Rows4 g1 = dbl_level1(P, L);
    const uint32_t B = g1.v[1], W = g1.v[2];
    const uint32_t E = mul_int<3>(g1.v[0]);  // 3 A                    m 3
    // L2: F = E^2 | C = B^2 | X B
    const Rows4 g2 = gather4(mul(sel4(L, E, B, P.X, P.X), sel4(L, E, B, B, B), L));
    const uint32_t C = g2.v[1], D = mul_int<4>(g2.v[2]);  // D = 4 X B       m 4
    const uint32_t X3 = sub<9>(g2.v[0], mul_int<2>(D), L);  // E^2 - 2 D   m 10
    const uint32_t t = sub<11>(D, X3, L);                   // D - X3      m 15
    // L3: E (D - X3), one product: every row computes it
    const uint32_t Y3 = sub<9>(mul(E, t, L), mul_int<8>(C), L);  // E (D - X3) - 8 C   m 10
    P.X = X3;
    P.Y = Y3;
    P.Z = mul_int<2>(W);  // 2 Y Z                                      m 2
}

// P = 2 P, and for the mixed addition of (x, y) that follows: ZZ = Z3^2, U2 = x ZZ, T = y Z3
__device__ __forceinline__ void dbl_zz(Pt& P, uint32_t x, uint32_t y, uint32_t& ZZ, uint32_t& U2, uint32_t& T,
                                       const Lane& L) {
    const Rows4 g1 = dbl_level1(P, L);
    const uint32_t B = g1.v[1], W = g1.v[2];
    const uint32_t E = mul_int<3>(g1.v[0]);
    // L2: F = E^2 | C = B^2 | X B | W^2
    const Rows4 g2 = gather4(mul(sel4(L, E, B, P.X, W), sel4(L, E, B, B, W), L));
    const uint32_t C = g2.v[1], D = mul_int<4>(g2.v[2]);
    const uint32_t X3 = sub<9>(g2.v[0], mul_int<2>(D), L);
    const uint32_t t = sub<11>(D, X3, L);
    const uint32_t Z3 = mul_int<2>(W);
    ZZ = mul_int<4>(g2.v[3]);  // (2 W)^2                              m 4
    // L3: E (D - X3) | x ZZ | y Z3
    const Rows4 g3 = gather4(mul(sel4(L, E, x, y, y), sel4(L, t, ZZ, Z3, Z3), L));
    P.X = X3;
    P.Y = sub<9>(g3.v[0], mul_int<8>(C), L);
    P.Z = Z3;
    U2 = g3.v[1];
    T = g3.v[2];
}

// P = P + (x, y) after dbl_zz (S2 = T ZZ = y Z^3)
__device__ __forceinline__ void madd_zz(Pt& P, uint32_t ZZ, uint32_t U2, uint32_t T, const Lane& L) {
    const uint32_t H = sub<11>(U2, P.X, L);  // U2 - X1                    m 12
    // La: HH = H^2 | S2 = T ZZ | Z H
    const Rows4 ga = gather4(mul(sel4(L, H, T, P.Z, P.Z), sel4(L, H, ZZ, H, H), L));
    const uint32_t I = mul_int<4>(ga.v[0]);        // 4 HH              m 4
    const uint32_t rr = sub<11>(ga.v[1], P.Y, L);  // S2 - Y1 = r / 2   m 12
    // Lb: J = H I | V = X I | rr^2
    const Rows4 gb = gather4(mul(sel4(L, H, P.X, rr, rr), sel4(L, I, I, rr, rr), L));
    const uint32_t J = gb.v[0], V = gb.v[1];
    uint32_t X3 = sub<2>(mul_int<4>(gb.v[2]), J, L);  // r^2 - J         m 6
    X3 = sub<3>(X3, mul_int<2>(V), L);                // - 2 V           m 9
    const uint32_t u = sub<10>(V, X3, L);             // V - X3          m 11
    // Lc: rr (V - X3) | Y J
    uint32_t ya, yb;
    gather01(mul(sel4(L, rr, P.Y, P.Y, P.Y), sel4(L, u, J, J, J), L), ya, yb);
    P.X = X3;
    P.Y = mul_int<2>(sub<2>(ya, yb, L));  // r (V - X3) - 2 Y1 J       m 6
    P.Z = mul_int<2>(ga.v[2]);             // 2 Z1 H                   m 2
}

// k (phi ? lambda : 1) P for the top 4 W bits of k held in SGPRs (k.v[0..3], wave-uniform; W = 32: a
// 128-bit k, W = 16: a 64-bit k in k.v[2..3] with k.v[0..1] = 0) over the co-Z table tab[8][3][16] (x, y,
// beta x of 1P .. 8P as row limbs of magnitude <= 1, lanes 10..15 zero): the trio kernel's radix-16
// Booth windows (the top digit = bit 127, then W windows of 4 doublings and one addition), neg
// negating every digit.  The digits, the infinity flag and every branch are wave-uniform.  Returns false
// when the result is infinity.
template <int W>
__device__ __forceinline__ bool glv_chain(Pt& acc, fe& k, bool neg, bool phi, const uint32_t* tab, const Lane& L) {
    const uint32_t one = L.one;
    bool inf = true;
    int d = static_cast<int>(k.v[3] >> 31);
    if (d != 0) {
        acc.X = tab[(phi ? 32 : 0) + L.k];
        acc.Y = tab[16 + L.k];
        if (neg) acc.Y = frow::neg<2>(acc.Y, L);
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
        if ((d < 0) != neg) y = frow::neg<2>(y, L);
        if (inf) {
            if (d != 0) {
                acc.X = x;
                acc.Y = y;
                acc.Z = one;
                inf = false;
            }
            continue;
        }
        dbl(acc, L);
        dbl(acc, L);
        dbl(acc, L);
        if (d != 0) {
            uint32_t ZZ, U2, T;
            dbl_zz(acc, x, y, ZZ, U2, T, L);
            madd_zz(acc, ZZ, U2, T, L);
        } else {
            dbl(acc, L);
        }
    }
    return !inf;
}

// ------------------------------------------------------------------ levels, conversions, tables
// one product level with a product per row: every row receives all four
__device__ __forceinline__ Rows4 level(const Lane& L, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                                       uint32_t b2, uint32_t a3, uint32_t b3) {
    return gather4(mul(sel4(L, a0, a1, a2, a3), sel4(L, b0, b1, b2, b3), L));
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
__device__ __forceinline__ void add_inc(Pt& R, const Pt& P, const Pt& Q, const Lane& L, uint32_t* Ho = nullptr,
                                        uint32_t* rro = nullptr) {
    const Rows4 g1 = level(L, P.Z, P.Z, Q.Z, Q.Z, P.Y, Q.Z, Q.Y, P.Z);  // Z1Z1 | Z2Z2 | Y1 Z2 | Y2 Z1
    const Rows4 g2 = level(L, P.X, g1.v[1], Q.X, g1.v[0], g1.v[2], g1.v[1], g1.v[3], g1.v[0]);  // U1 | U2 | S1 | S2
    const uint32_t U1 = g2.v[0], S1 = g2.v[2];
    const uint32_t H = sub<2>(g2.v[1], U1, L);              // U2 - U1          m 3
    const uint32_t t = mul_int<2>(H);                       // 2 H              m 6
    const uint32_t rr = mul_int<2>(sub<2>(g2.v[3], S1, L));  // 2 (S2 - S1)      m 6
    const Rows4 g3 = level(L, t, t, rr, rr, P.Z, Q.Z, P.Z, Q.Z);  // I = (2H)^2 | rr^2 | Z1 Z2
    const uint32_t I = g3.v[0];
    const Rows4 g4 = level(L, H, I, U1, I, g3.v[2], H, g3.v[2], H);  // J = H I | V = U1 I | Z1 Z2 H
    const uint32_t J = g4.v[0], V = g4.v[1];
    uint32_t X3 = sub<2>(g3.v[1], J, L);  // rr^2 - J                             m 3
    X3 = sub<3>(X3, mul_int<2>(V), L);    // - 2 V                                m 6
    const uint32_t u = sub<7>(V, X3, L);  // V - X3                               m 8
    uint32_t ya, yb;
    gather01(mul(sel4(L, rr, S1, S1, S1), sel4(L, u, J, J, J), L), ya, yb);
    R.X = X3;
    R.Y = sub<3>(ya, mul_int<2>(yb), L);  // rr (V - X3) - 2 S1 J                m 4
    R.Z = mul_int<2>(g4.v[2]);            // 2 Z1 Z2 H                           m 2
    if (Ho) *Ho = H;
    if (rro) *rro = rr;
}

// R = P + Q, complete: infinity on either side, P = Q (doubling), P = -Q (infinity) -- ec26.h's cases.
// Every flag and test is wave-uniform.
__device__ __forceinline__ void add_full(Pt& R, bool& rinf, const Pt& P, bool pinf, const Pt& Q, bool qinf,
                                         uint32_t* slot, const Lane& L) {
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
    add_inc(S, P, Q, L, &H, &rr);
    rinf = false;
    if (is_zero(H, slot, L)) {
        if (is_zero(rr, slot, L)) {
            S = P;
            dbl(S, L);
        } else {
            rinf = true;
        }
    }
    R = S;
}

// P = P + (x, y), (x, y) affine m <= 2, P != +-(x, y), P not at infinity: 5 levels -> (9, 6, 2)
__device__ __forceinline__ void madd(Pt& P, uint32_t x, uint32_t y, const Lane& L) {
    uint32_t ZZ, T;
    gather01(mul(sel4(L, P.Z, y, y, y), sel4(L, P.Z, P.Z, P.Z, P.Z), L), ZZ, T);  // Z^2 | y Z
    const uint32_t U2 = mul(x, ZZ, L);                                           // (every row)
    madd_zz(P, ZZ, U2, T, L);
}

// The GLV table of a point P1 (Jacobian, magnitudes <= 16, of order n): 1P .. 8P rescaled to the common
// Zc = Z1 ... Z8 (entries affine on the curve y^2 = x^3 + 7 Zc^6 w^3, as coz_table26) -> tab[j][0] = x,
// tab[j][1] = y, tab[j][2] = beta x (row limbs, magnitude 1), zc = Zc.  The additions never meet
// P = +-Q (jP +- P for j <= 6 and P of order n); an invalid P only yields a table whose verdict is
// already false.
__device__ __forceinline__ void build_table(uint32_t (*tab)[3][16], uint32_t* zc, const Pt& P1, uint32_t beta,
                                            const Lane& L) {
    Pt T[8];
    T[0] = P1;
    T[1] = P1;
    dbl(T[1], L);
    add_inc(T[2], T[1], T[0], L);
    T[3] = T[1];
    dbl(T[3], L);
    add_inc(T[4], T[3], T[0], L);
    T[5] = T[2];
    dbl(T[5], L);
    add_inc(T[6], T[5], T[0], L);
    T[7] = T[3];
    dbl(T[7], L);
    // prefix and suffix products of the Z's, side by side (rows 0 / 1)
    uint32_t pre[8], suf[8];
    pre[0] = T[0].Z;
    suf[7] = T[7].Z;
#pragma unroll
    for (int j = 1; j < 8; ++j)
        gather01(mul(sel4(L, pre[j - 1], suf[8 - j], suf[8 - j], suf[8 - j]),
                     sel4(L, T[j].Z, T[7 - j].Z, T[7 - j].Z, T[7 - j].Z), L),
                 pre[j], suf[7 - j]);
    // s_j = Zc / Z_j = pre_(j-1) suf_(j+1)
    uint32_t sj[8], s2[8], s3[8], xs[8];
    sj[0] = suf[1];
    sj[7] = pre[6];
    {
        const Rows4 g = level(L, pre[0], suf[2], pre[1], suf[3], pre[2], suf[4], pre[3], suf[5]);
        sj[1] = g.v[0];
        sj[2] = g.v[1];
        sj[3] = g.v[2];
        sj[4] = g.v[3];
        uint32_t a, b;
        gather01(mul(sel4(L, pre[4], pre[5], pre[5], pre[5]), sel4(L, suf[6], suf[7], suf[7], suf[7]), L), a, b);
        sj[5] = a;
        sj[6] = b;
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
        const Rows4 g = level(L, sj[j], sj[j], sj[j + 1], sj[j + 1], sj[j + 2], sj[j + 2], sj[j + 3], sj[j + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) s2[j + q] = g.v[q];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {  // s^3 and X s^2 of two entries per level
        const Rows4 g = level(L, s2[j], sj[j], T[j].X, s2[j], s2[j + 1], sj[j + 1], T[j + 1].X, s2[j + 1]);
        s3[j] = g.v[0];
        xs[j] = g.v[1];
        s3[j + 1] = g.v[2];
        xs[j + 1] = g.v[3];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {  // Y s^3
        const Rows4 g = level(L, T[j].Y, s3[j], T[j + 1].Y, s3[j + 1], T[j + 2].Y, s3[j + 2], T[j + 3].Y, s3[j + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (L.row == 0 && L.k < 16) tab[j + q][1][L.k] = g.v[q];
    }
#pragma unroll
    for (int j = 0; j < 8; j += 4) {  // beta x
        const Rows4 g = level(L, beta, xs[j], beta, xs[j + 1], beta, xs[j + 2], beta, xs[j + 3]);
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
__device__ __forceinline__ uint32_t sqr_n(uint32_t a, int n, const Lane& L) {
    uint32_t t = sqr(a, L);
#pragma unroll 1
    for (int i = 1; i < n; ++i) t = sqr(t, L);
    return t;
}
__device__ __forceinline__ uint32_t sqrt_cand(uint32_t a, const Lane& L) {
    const uint32_t x2 = mul(sqr(a, L), a, L);
    const uint32_t x3 = mul(sqr(x2, L), a, L);
    const uint32_t x6 = mul(sqr_n(x3, 3, L), x3, L);
    const uint32_t x9 = mul(sqr_n(x6, 3, L), x3, L);
    const uint32_t x11 = mul(sqr_n(x9, 2, L), x2, L);
    const uint32_t x22 = mul(sqr_n(x11, 11, L), x11, L);
    const uint32_t x44 = mul(sqr_n(x22, 22, L), x22, L);
    const uint32_t x88 = mul(sqr_n(x44, 44, L), x44, L);
    const uint32_t x176 = mul(sqr_n(x88, 88, L), x88, L);
    const uint32_t x220 = mul(sqr_n(x176, 44, L), x44, L);
    const uint32_t x223 = mul(sqr_n(x220, 3, L), x3, L);
    uint32_t t = mul(sqr_n(x223, 23, L), x22, L);
    t = mul(sqr_n(t, 6, L), x2, L);
    return sqr_n(t, 2, L);
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
