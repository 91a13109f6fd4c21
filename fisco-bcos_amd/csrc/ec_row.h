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

// k (phi ? lambda : 1) R' for a 128-bit k held in SGPRs (k.v[0..3], wave-uniform) over the co-Z table
// tab[8][3][16] (x, y, beta x of 1R' .. 8R' as canonical limbs, lanes 10..15 zero): the trio kernel's
// 33 radix-16 Booth windows (digit 32 = bit 127, then 32 windows of 4 doublings and one addition),
// neg negating every digit.  The digits, the infinity flag and every branch are wave-uniform.
// Returns false when the result is infinity.
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
    for (int w = 31; w >= 0; --w) {
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

}  // namespace frow
}  // namespace bcosgpu
