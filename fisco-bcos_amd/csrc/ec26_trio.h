// ec26_trio.h -- secp256k1 point doubling and mixed addition split over a lane TRIO: three adjacent
// lanes of one wave (positions 3t, 3t + 1, 3t + 2 of a 16-lane DPP row; position 15 is a phantom
// role-0 lane whose results are never used) cooperate on ONE point, each lane computing one of the
// independent field multiplications of a dependency level.  Operands are routed between the lanes of
// a trio by DPP row shifts (row_shr / row_shl by 1 or 2) and per-role selects, so a level costs one
// multiplication of latency and no barrier and no LDS round trip -- the wave-pair split of
// coop26_dbl / coop26_madd (ecc_coop.hip) paid a __syncthreads and an LDS write + read per level.
//
// Every lane executes the same instruction stream (a wave has one program counter): a level is one
// fe26_mul / fe26_sqr whose operands are chosen per role, so the split must give all roles the same
// operation at each level.  The formulas are CurveK1x's (ec26.h) with the same magnitudes:
//
//   dbl (3 levels):  L1  A = X^2          | B = Y^2            | B = Y^2   (redundant)
//                    L2  F = (3A)^2       | C = B^2            | XB = X B
//                    L3  --               | E (D - X3)         | Y Z       (lane 1 gathers E, F, XB)
//                    D = 4 XB, X3 = F - 2D, Y3 = E (D - X3) - 8C, Z3 = 2 Y Z
//   madd (5 levels): L1  Z^2              | y2 Z               | Z^2
//                    L2  U2 = x2 Z^2      | S2 = y2 Z Z^2      | U2
//                    L3  HH = H^2         | rr^2               | Z H       (H = U2 - X, rr = S2 - Y)
//                    L4  J = H I          | --                 | V = X I   (I = 4 HH)
//                    L5  rr (V - X3)      | Y J                | --
//                    X3 = 4 rr^2 - J - 2V, Y3 = 2 (rr (V - X3) - Y J), Z3 = 2 Z H
//
// A point lives in the trio as TrioPt: S1 = (X | Y | Y) (the first doubling level's operand), Xs = X
// and Zs = Z on lane 2 (lanes 0 and 1 hold don't-care values there), inf on every lane.  Magnitudes:
// dbl -> (10, 10, 2), madd -> (9, 6, 2), as CurveK1x.
#pragma once
#include "ec26.h"

#ifndef TRIO_DUMP  // tools/triobench.hip defines it to dump the addition's per-level values
#define TRIO_DUMP(slot, a) ((void)0)
#endif

namespace bcosgpu {

struct TrioPt {
    fe26 S1, Xs, Zs;
    bool inf;
};

// lane role inside its trio, the three role predicates and (device) their wave masks for
// v_cndmask_b32_dpp (n* = complements)
struct TrioLane {
    bool r0, r1, r2;
    uint64_t m0, m1, m2, n0, n1, n2;
    F26_HD explicit TrioLane(int lane) {
        const int role = (lane & 15) % 3;
        r0 = role == 0;
        r1 = role == 1;
        r2 = role == 2;
#if defined(__HIP_DEVICE_COMPILE__)
        m0 = __builtin_amdgcn_ballot_w64(r0);
        m1 = __builtin_amdgcn_ballot_w64(r1);
        m2 = __builtin_amdgcn_ballot_w64(r2);
#else
        m0 = m1 = m2 = 0;
#endif
        n0 = ~m0;
        n1 = ~m1;
        n2 = ~m2;
    }
};

#if !defined(__HIP_DEVICE_COMPILE__)
// host emulation of a DPP row (tests/cpp/trio_test.cpp runs the 16 lanes of a row as threads)
uint32_t trio_emu_dpp(uint32_t x, int ctrl);
bool trio_emu_any(bool b);
#endif

namespace trio {
// DPP fetches inside a 16-lane row: L1 / L2 = the value of lane i - 1 / i - 2 (row_shr), R1 / R2 = of
// lane i + 1 / i + 2 (row_shl); out-of-row sources read 0 (bound_ctrl), which only phantom lanes see
template <int CTRL>
F26_HD uint32_t dpp(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, 0xf, 0xf, true));
#else
    return trio_emu_dpp(x, CTRL);
#endif
}
F26_HD bool any(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __any(b);
#else
    return trio_emu_any(b);
#endif
}
constexpr int kL1 = 0x111, kL2 = 0x112, kR1 = 0x101, kR2 = 0x102;

// the magnitude of a fetched element travels with it in the checking build (a phantom lane's zero
// reads as magnitude 1)
#ifdef FE26_CHECK
template <int CTRL>
F26_HD int mdpp(int m) {
    const int r = static_cast<int>(dpp<CTRL>(static_cast<uint32_t>(m)));
    return r ? r : 1;
}
#endif

template <int CTRL, class E>
F26_HD void fdpp(E& r, const E& a) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = dpp<CTRL>(a.v[i]);
    F26_SETM(r, mdpp<CTRL>(a.m));
}
// A DPP read needs two wait states after the VALU write of its source VGPR (gfx9 rule).  The compiler
// pads its own code, but not the boundary after an inline-asm block (fe26_mul_asm / fe26_sqr_asm end
// with VALU writes of their result limbs; fp26_mul_asm / fp26_sqr_asm likewise), so every product a
// lane may fetch goes through these: the
// s_nop names the limbs as in/out operands, so any later DPP read of them is ordered after it.
template <class E>
F26_HD void dpp_fence(E& r) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("s_nop 1"
                 : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
                   "+v"(r.v[6]), "+v"(r.v[7]), "+v"(r.v[8]), "+v"(r.v[9]));
#else
    (void)r;
#endif
}
F26_HD void mul(fe26& r, const fe26& a, const fe26& b) {
    fe26_mul(r, a, b);
    dpp_fence(r);
}
F26_HD void sqr(fe26& r, const fe26& a) {
    fe26_sqr(r, a);
    dpp_fence(r);
}
template <class E>
F26_HD void sel(E& r, bool c, const E& a, const E& b) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    F26_SETM(r, c ? a.m : b.m);
}
// c ? a : (d ? DPP<C1>(b) : DPP<C2>(b))
template <int C1, int C2, class E>
F26_HD void sel_dpp2(E& r, bool c, const E& a, bool d, const E& b) {
#ifdef FE26_CHECK
    const int m1 = mdpp<C1>(b.m), m2 = mdpp<C2>(b.m);
#endif
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t x = dpp<C1>(b.v[i]), y = dpp<C2>(b.v[i]);
        r.v[i] = c ? a.v[i] : (d ? x : y);
    }
    F26_SETM(r, c ? a.m : d ? m1 : m2);
}
// r = c ? a : DPP<CTRL>(b) in one v_cndmask_b32_dpp per limb (the DPP combiner is off, so the fold
// is written out): VCC = cm, the wave mask of c; s_nop 1 gives the DPP source its two wait states
// after a VALU write (SALU -> VALU reads of VCC need none).  Five limbs per block (operand limit).
#define TRIO_CSEL_INS(D, S0, S1, CTL) "v_cndmask_b32_dpp %" #D ", %" #S0 ", %" #S1 ", vcc " CTL \
    " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define TRIO_CSEL5(CTL, r, a, b, o, cm)                                                                \
    asm volatile("s_mov_b64 vcc, %15\n\ts_nop 1\n\t" TRIO_CSEL_INS(0, 10, 5, CTL) TRIO_CSEL_INS(1, 11, 6, CTL) \
                 TRIO_CSEL_INS(2, 12, 7, CTL) TRIO_CSEL_INS(3, 13, 8, CTL) TRIO_CSEL_INS(4, 14, 9, CTL)      \
                 : "=&v"((r).v[o]), "=&v"((r).v[o + 1]), "=&v"((r).v[o + 2]), "=&v"((r).v[o + 3]),       \
                   "=&v"((r).v[o + 4])                                                                  \
                 : "v"((a).v[o]), "v"((a).v[o + 1]), "v"((a).v[o + 2]), "v"((a).v[o + 3]), "v"((a).v[o + 4]), \
                   "v"((b).v[o]), "v"((b).v[o + 1]), "v"((b).v[o + 2]), "v"((b).v[o + 3]), "v"((b).v[o + 4]), \
                   "s"(cm)                                                                              \
                 : "vcc")
template <int CTRL, class E>
F26_HD void csel(E& r, bool c, uint64_t cm, const E& a, const E& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    (void)c;
    E t;
    if constexpr (CTRL == kL1) {
        TRIO_CSEL5("row_shr:1", t, a, b, 0, cm);
        TRIO_CSEL5("row_shr:1", t, a, b, 5, cm);
    } else if constexpr (CTRL == kL2) {
        TRIO_CSEL5("row_shr:2", t, a, b, 0, cm);
        TRIO_CSEL5("row_shr:2", t, a, b, 5, cm);
    } else if constexpr (CTRL == kR1) {
        TRIO_CSEL5("row_shl:1", t, a, b, 0, cm);
        TRIO_CSEL5("row_shl:1", t, a, b, 5, cm);
    } else {
        static_assert(CTRL == kR2, "csel: row shift by 1 or 2");
        TRIO_CSEL5("row_shl:2", t, a, b, 0, cm);
        TRIO_CSEL5("row_shl:2", t, a, b, 5, cm);
    }
    r = t;
#else
    (void)cm;
#ifdef FE26_CHECK
    const int mb = mdpp<CTRL>(b.m);
#endif
    E t;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t x = dpp<CTRL>(b.v[i]);
        t.v[i] = c ? a.v[i] : x;
    }
    F26_SETM(t, c ? a.m : mb);
    r = t;
#endif
}
F26_HD uint32_t bdpp_from(uint32_t f, const TrioLane& T, int src) {
    // the value of f held by role src of this lane's trio
    const uint32_t l1 = dpp<kL1>(f), l2 = dpp<kL2>(f), r1 = dpp<kR1>(f), r2 = dpp<kR2>(f);
    if (src == 0) return T.r0 ? f : T.r1 ? l1 : l2;
    if (src == 1) return T.r1 ? f : T.r0 ? r1 : l1;
    return T.r2 ? f : T.r1 ? r1 : r2;
}
}  // namespace trio

F26_HD void trio_from_aff(TrioPt& P, const Aff26& Q, const TrioLane& T) {
    trio::sel(P.S1, T.r0, Q.x, Q.y);
    fe26_copy(P.Xs, Q.x);
    fe26_one(P.Zs);
    P.inf = false;
}
F26_HD void trio_set_inf(TrioPt& P) {
    fe26_zero(P.S1);
    fe26_zero(P.Xs);
    fe26_zero(P.Zs);
    P.inf = true;
}
F26_HD void trio_cmov(TrioPt& P, const TrioPt& Q, bool c) {
    fe26_cmov(P.S1, Q.S1, c);
    fe26_cmov(P.Xs, Q.Xs, c);
    fe26_cmov(P.Zs, Q.Zs, c);
    P.inf = c ? Q.inf : P.inf;
}
// the full Jacobian point on every lane of the trio (X from lane 0, Y from lane 1, Z from lane 2)
F26_HD void trio_to_jac(Jac26& J, const TrioPt& P, const TrioLane& T) {
    using namespace trio;
    sel_dpp2<kL1, kL2>(J.X, T.r0, P.S1, T.r1, P.S1);   // lane 1 <- lane 0, lane 2 <- lane 0
    sel_dpp2<kR1, kL1>(J.Y, T.r1, P.S1, T.r0, P.S1);   // lane 0 <- lane 1, lane 2 <- lane 1
    sel_dpp2<kR1, kR2>(J.Z, T.r2, P.Zs, T.r1, P.Zs);   // lane 1 <- lane 2, lane 0 <- lane 2
    J.inf = P.inf;
}

// P <- 2P  (X, Y <= 10, Z <= 16 -> (10, 10, 2))
F26_HD void trio_dbl(TrioPt& P, const TrioLane& T) {
    using namespace trio;
    fe26 o1, T2, S2, o2, F, XB, D, X3, W, P3, Q3, o3, C8, Y3, t;
    sqr(o1, P.S1);                                       // (A | B | B)                 m 1
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t x3 = (o1.v[i] << 1) + o1.v[i];  // one v_lshl_add_u32
        T2.v[i] = T.r0 ? x3 : o1.v[i];                  // (3A | B | B)               m <= 3
    }
    F26_SETM(T2, T.r0 ? 3 : 1);
    sel(S2, T.r2, P.Xs, T2);                             // (3A | B | X)                m <= 10
    mul(o2, S2, T2);                                     // (F | C | XB)
    fdpp<kL1>(F, o2);                                    // lane 1: F                   m 1
    fdpp<kR1>(XB, o2);                                   // lane 1: X B                 m 1
    fe26_mul_int<4>(D, XB);                              // D = 4 X B                   m 4
    fe26_mul_int<2>(t, D);                               //                             m 8
    fe26_sub<9>(X3, F, t);                               // X3 = F - 2D                 m 10
    fe26_sub<11>(W, D, X3);                              // D - X3                      m 15
    csel<kL1>(P3, T.r2, T.m2, P.S1, T2);                 // lane 1: E = 3A (lane 0), lane 2: Y
    sel(Q3, T.r2, P.Zs, W);                              // lane 1: D - X3, lane 2: Z
    mul(o3, P3, Q3);                                     // (- | E (D - X3) | Y Z)
    fe26_mul_int<8>(C8, o2);                             // lane 1: 8C                  m 8
    fe26_sub<9>(Y3, o3, C8);                             // lane 1: Y3                  m 10
    fe26_mul_int<2>(P.Zs, o3);                           // lane 2: Z3 = 2 Y Z          m 2
    // next state: S1 = (X3 | Y3 | Y3) from lane 1, Xs = X3 on lane 2
    csel<kL1>(t, T.r1, T.m1, Y3, Y3);                    // lanes 1, 2: Y3 of lane 1
    csel<kR1>(P.S1, !T.r0, T.n0, t, X3);                 // lane 0: X3 of lane 1
    fdpp<kL1>(P.Xs, X3);                                 // lane 2 <- X3 of lane 1
}

// R <- P + Q, Q affine (x, y <= 2) and never infinity; P: X, Y <= 10, Z <= 16 -> (9, 6, 2).  The
// exceptional cases are those of CurveK1x::madd: P = Q doubles (computed on lane 2, which holds all of
// P), P = -Q gives infinity, P = infinity gives Q.  EXC = false drops the P = +-Q tests for callers
// that exclude those cases (trio_add_digit in ecc_coop.hip states why a GLV chain does).
template <bool EXC = true>
F26_HD void trio_madd(TrioPt& R, const TrioPt& P, const Aff26& Q, const TrioLane& T) {
    using namespace trio;
    fe26 Zb, P1, o1, P2, Q2, o2, Xl, h, P3, o3, HHx, I, P4, o4, R2, V, X3, W, P5, Q5, o5, Y3, t;
    sel_dpp2<kR1, kR2>(Zb, T.r2, P.Zs, T.r1, P.Zs);     // Z on every lane
    sel(P1, T.r1, Q.y, Zb);
    mul(o1, P1, Zb);                                     // (Z1Z1 | y2 Z | Z1Z1)
    TRIO_DUMP(0, o1);
    sel(P2, T.r1, o1, Q.x);
    fdpp<kR1>(Q2, o1);
    sel(Q2, T.r1, Q2, o1);                               // lane 1: Z1Z1 of lane 2
    mul(o2, P2, Q2);                                     // (U2 | S2 | U2)
    TRIO_DUMP(1, o2);
    sel(Xl, T.r2, P.Xs, P.S1);                           // (X | Y | X)                 m <= 10
    fe26_sub<11>(h, o2, Xl);                             // (H | rr | H)                m 12
    sel(P3, T.r2, Zb, h);
    mul(o3, P3, h);                                      // (HH | rr^2 | Z H)
    TRIO_DUMP(2, h);
    TRIO_DUMP(3, o3);
    fdpp<kL2>(HHx, o3);
    sel(HHx, T.r2, HHx, o3);                             // lanes 0, 2: HH
    fe26_mul_int<4>(I, HHx);                             // I = 4 HH                    m 4
    sel(P4, T.r2, P.Xs, h);
    mul(o4, P4, I);                                      // (J | - | V)
    TRIO_DUMP(4, o4);
    // lane 0: X3 = 4 rr^2 - J - 2V and V - X3
    fdpp<kR1>(R2, o3);
    fe26_mul_int<4>(R2, R2);                             // 4 rr^2                      m 4
    fdpp<kR2>(V, o4);                                    // V of lane 2                 m 1
    fe26_sub<2>(X3, R2, o4);                             //                             m 6
    fe26_mul_int<2>(t, V);                               //                             m 2
    fe26_sub<3>(X3, X3, t);                              // X3                          m 9
    fe26_sub<10>(W, V, X3);                              // V - X3                      m 11
    fdpp<kR1>(P5, h);
    sel(P5, T.r0, P5, P.S1);                             // lane 0: rr (lane 1), lane 1: Y   m 12
    fdpp<kL1>(Q5, o4);
    sel(Q5, T.r0, W, Q5);                                // lane 0: V - X3, lane 1: J of lane 0
    mul(o5, P5, Q5);                                     // (rr (V - X3) | Y J | -)
    TRIO_DUMP(5, o5);
    TRIO_DUMP(6, X3);
    fdpp<kR1>(t, o5);
    fe26_sub<2>(Y3, o5, t);                              //                             m 3
    fe26_mul_int<2>(Y3, Y3);                             // lane 0: Y3                  m 6
    TRIO_DUMP(7, Y3);
    TrioPt O;
    sel_dpp2<kL1, kL2>(O.S1, T.r0, X3, T.r1, Y3);      // (X3 | Y3 | Y3) from lane 0
    fdpp<kL2>(O.Xs, X3);                                 // lane 2 <- X3 of lane 0
    fe26_mul_int<2>(O.Zs, o3);                           // lane 2: Z3 = 2 Z H          m 2
    O.inf = false;
    if constexpr (EXC) {  // exceptional cases (flags shared across the trio)
        const uint32_t zf = fe26_is_zero(h) ? 1u : 0u;
        const bool hz = bdpp_from(zf, T, 0) != 0u && !P.inf;
        const bool rz = bdpp_from(zf, T, 1) != 0u;
        if (any(hz && rz)) {                             // P == Q: double on lane 2 (rare)
            Jac26 A, D;
            fe26_copy(A.X, P.Xs);
            fe26_copy(A.Y, P.S1);
            fe26_copy(A.Z, P.Zs);
            A.inf = P.inf;
            CurveK1x::dbl(D, A);
            TrioPt Dt;
            sel_dpp2<kR2, kR1>(Dt.S1, T.r2, D.Y, T.r0, D.X);  // lane 0 <- X, lane 1 <- Y of lane 2
#pragma unroll
            for (int i = 0; i < 10; ++i) {
                const uint32_t y = dpp<kR1>(D.Y.v[i]);
                Dt.S1.v[i] = T.r1 ? y : Dt.S1.v[i];
            }
            F26_SETM(Dt.S1, 10);
            fe26_copy(Dt.Xs, D.X);
            fe26_copy(Dt.Zs, D.Z);
            Dt.inf = false;
            trio_cmov(O, Dt, hz && rz);
        }
        if (hz && !rz) O.inf = true;                     // P == -Q
    }
    if (P.inf) trio_from_aff(O, Q, T);
    R = O;
}

// P <- 2P as trio_dbl, and ZZ = Z3^2 on lane 0 for the mixed addition that follows (trio_madd_zz): the
// first level's redundant lane-2 square becomes Z^2 (lane 2's B comes from lane 1), and the third
// level's idle lane 0 computes B Z^2, so Z3^2 = (2 Y Z)^2 = 4 B Z^2 costs no product level.
// (X, Y <= 10, Z <= 16 -> (10, 10, 2), ZZ m 4)
F26_HD void trio_dbl_zz(TrioPt& P, fe26& ZZ, const TrioLane& T) {
    using namespace trio;
    fe26 S0, o1, T2, S2, o2, F, XB, D, X3, W, P3, Q3, o3, C8, Y3, t;
    sel(S0, T.r2, P.Zs, P.S1);                           // (X | Y | Z)
    sqr(o1, S0);                                         // (A | B | Z^2)                m 1
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t x3 = (o1.v[i] << 1) + o1.v[i];  // one v_lshl_add_u32
        T2.v[i] = T.r0 ? x3 : o1.v[i];                  // (3A | B | Z^2)
    }
    F26_SETM(T2, T.r0 ? 3 : 1);
    csel<kL1>(T2, !T.r2, T.n2, T2, o1);                  // lane 2: B of lane 1 -> (3A | B | B)
    sel(S2, T.r2, P.Xs, T2);                             // (3A | B | X)                 m <= 10
    mul(o2, S2, T2);                                     // (F | C | XB)
    fdpp<kL1>(F, o2);                                    // lane 1: F                    m 1
    fdpp<kR1>(XB, o2);                                   // lane 1: X B                  m 1
    fe26_mul_int<4>(D, XB);                              // D = 4 X B                    m 4
    fe26_mul_int<2>(t, D);                               //                              m 8
    fe26_sub<9>(X3, F, t);                               // X3 = F - 2D                  m 10
    fe26_sub<11>(W, D, X3);                              // D - X3                       m 15
    csel<kL1>(P3, T.r2, T.m2, P.S1, T2);                 // lane 1: E = 3A (lane 0), lane 2: Y
    csel<kR1>(P3, !T.r0, T.n0, P3, o1);                  // lane 0: B (lane 1)
    sel(Q3, T.r2, P.Zs, W);                              // lane 1: D - X3, lane 2: Z
    csel<kR2>(Q3, !T.r0, T.n0, Q3, o1);                  // lane 0: Z^2 (lane 2)
    mul(o3, P3, Q3);                                     // (B Z^2 | E (D - X3) | Y Z)
    fe26_mul_int<4>(ZZ, o3);                             // lane 0: Z3^2 = 4 B Z^2       m 4
    fe26_mul_int<8>(C8, o2);                             // lane 1: 8C                   m 8
    fe26_sub<9>(Y3, o3, C8);                             // lane 1: Y3                   m 10
    fe26_mul_int<2>(P.Zs, o3);                           // lane 2: Z3 = 2 Y Z           m 2
    csel<kL1>(t, T.r1, T.m1, Y3, Y3);                    // lanes 1, 2: Y3 of lane 1
    csel<kR1>(P.S1, !T.r0, T.n0, t, X3);                 // lane 0: X3 of lane 1
    fdpp<kL1>(P.Xs, X3);                                 // lane 2 <- X3 of lane 1
}

// R <- P + Q, Q affine, given ZZ = Z1^2 on lane 0 (trio_dbl_zz): CurveK1x::madd in 4 product levels
// instead of 5 (the Z1^2 level is gone), without the P = +-Q tests (the GLV chain's additions, see
// trio_add_digit in ecc_coop.hip); P = infinity gives Q.  X, Y <= 10, Z <= 16, ZZ <= 4; Q <= 2
// -> (9, 6, 2).
//   L1  U2 = x2 ZZ       | T = y2 Z        | --
//   L2  HH = H^2         | S2 = T ZZ       | Z H          (H = U2 - X on lane 0)
//   L3  J = H I          | rr^2            | V = X I      (I = 4 HH, rr = S2 - Y on lane 1)
//   L4  rr (V - X3)      | Y J             | --           (X3 = 4 rr^2 - J - 2V on lane 0)
F26_HD void trio_madd_zz(TrioPt& R, const TrioPt& P, const fe26& ZZ, const Aff26& Q, const TrioLane& T) {
    using namespace trio;
    fe26 P1, Q1, o1, h, P2, Q2, a, b, o2, I, rr, P3, Q3, o3, R2, V, X3, W, P4, Q4, o4, Y3, t;
    sel(P1, T.r1, Q.y, Q.x);                             // (x2 | y2 | x2)
    csel<kR1>(Q1, T.r0, T.m0, ZZ, P.Zs);                 // (ZZ | Z of lane 2 | -)
    mul(o1, P1, Q1);                                     // (U2 | T | -)
    fe26_sub<11>(h, o1, P.S1);                           // lane 0: H = U2 - X           m 12
    sel(P2, T.r1, o1, P.Zs);
    sel(P2, T.r0, h, P2);                                // (H | T | Z)
    fdpp<kL1>(a, ZZ);                                    // lane 1: ZZ
    fdpp<kL2>(b, h);                                     // lane 2: H
    sel(Q2, T.r1, a, b);
    sel(Q2, T.r0, h, Q2);                                // (H | ZZ | H)
    mul(o2, P2, Q2);                                     // (HH | S2 | Z H)
    fe26_mul_int<4>(I, o2);                              // lane 0: I = 4 HH             m 4
    fe26_sub<11>(rr, o2, P.S1);                          // lane 1: rr = S2 - Y          m 12
    sel(P3, T.r1, rr, P.Xs);
    sel(P3, T.r0, h, P3);                                // (H | rr | X)
    fdpp<kL2>(b, I);                                     // lane 2: I
    sel(Q3, T.r1, rr, b);
    sel(Q3, T.r0, I, Q3);                                // (I | rr | I)
    mul(o3, P3, Q3);                                     // (J | rr^2 | V)
    // lane 0: X3 = 4 rr^2 - J - 2V and V - X3
    fdpp<kR1>(R2, o3);
    fe26_mul_int<4>(R2, R2);                             // 4 rr^2                       m 4
    fdpp<kR2>(V, o3);                                    // V of lane 2                  m 1
    fe26_sub<2>(X3, R2, o3);                             //                              m 6
    fe26_mul_int<2>(t, V);                               //                              m 2
    fe26_sub<3>(X3, X3, t);                              // X3                           m 9
    fe26_sub<10>(W, V, X3);                              // V - X3                       m 11
    csel<kR1>(P4, !T.r0, T.n0, P.S1, rr);                // lane 0: rr (lane 1), lane 1: Y   m 12
    csel<kL1>(Q4, T.r0, T.m0, W, o3);                    // lane 0: V - X3, lane 1: J of lane 0
    mul(o4, P4, Q4);                                     // (rr (V - X3) | Y J | -)
    fdpp<kR1>(t, o4);
    fe26_sub<2>(Y3, o4, t);                              //                              m 3
    fe26_mul_int<2>(Y3, Y3);                             // lane 0: Y3                   m 6
    TrioPt O;
    sel_dpp2<kL1, kL2>(O.S1, T.r0, X3, T.r1, Y3);      // (X3 | Y3 | Y3) from lane 0
    fdpp<kL2>(O.Xs, X3);                                 // lane 2 <- X3 of lane 0
    fe26_mul_int<2>(O.Zs, o2);                           // lane 2: Z3 = 2 Z H           m 2
    O.inf = false;
    if (P.inf) trio_from_aff(O, Q, T);
    R = O;
}

// R <- P + Q, both Jacobian in trio form (lane 2 holds all of each point at entry); CurveK1x::add's
// formulas, magnitudes and exceptional cases (P = Q doubles on lane 2, P = -Q gives infinity, an
// infinite operand gives the other), 16 products in 6 levels:
//   L1  Z1Z1 = Z1^2      | Z2Z2 = Z2^2     | A = Y1 Z2
//   L2  U2 = X2 Z1Z1     | U1 = X1 Z2Z2    | B = Y2 Z1
//   L3  S2 = B Z1Z1      | S1 = A Z2Z2     | I = (2H)^2          (H = U2 - U1 on lane 2)
//   L4  J = H I          | V = U1 I        | r^2                 (r = 2 (S2 - S1) on lane 2)
//   L5  r (V - X3)       | S1 J            | Z1 Z2               (X3 = r^2 - J - 2V on lane 0)
//   L6  --               | --              | Z1 Z2 H
//   X3 = r^2 - J - 2V, Y3 = r (V - X3) - 2 S1 J, Z3 = 2 Z1 Z2 H.  X, Y, Z <= 16 (both) -> (6, 4, 2).
F26_HD void trio_add(TrioPt& R, const TrioPt& P, const TrioPt& Q, const TrioLane& T) {
    using namespace trio;
    fe26 a, b, P1, Q1, o1, P2, Q2, o2, u2, u1, h, h2, P3, Q3, o3, s2, s1, rr, P4, Q4, o4, rv, X3, W, P5, Q5, o5,
        Y3, Z3, t;
    // L1: lane 0 Z1 Z1 (Z1 of lane 2), lane 1 Z2 Z2 (Z2 of lane 2), lane 2 Y1 Z2
    fdpp<kR2>(a, P.Zs);                                  // lane 0: Z1
    fdpp<kR1>(b, Q.Zs);                                  // lane 1: Z2
    sel(P1, T.r0, a, b);
    sel(P1, T.r2, P.S1, P1);
    sel(Q1, T.r2, Q.Zs, P1);
    mul(o1, P1, Q1);                                     // (Z1Z1 | Z2Z2 | A)            m 1
    // L2: lane 0 X2 Z1Z1, lane 1 X1 Z2Z2 (X1 of lane 0), lane 2 Y2 Z1
    fdpp<kL1>(a, P.S1);                                  // lane 1: X1
    sel(P2, T.r1, a, Q.S1);                              // (X2 | X1 | Y2)
    sel(Q2, T.r2, P.Zs, o1);                             // (Z1Z1 | Z2Z2 | Z1)
    mul(o2, P2, Q2);                                     // (U2 | U1 | B)
    // lane 2: H = U2 - U1, 2H
    fdpp<kL2>(u2, o2);                                   // lane 0's U2 at lane 2
    fdpp<kL1>(u1, o2);                                   // lane 1's U1 at lane 2
    fe26_sub<2>(h, u2, u1);                              // H                            m 3
    fe26_mul_int<2>(h2, h);                              // 2H                           m 6
    // L3: lane 0 B Z1Z1 (B of lane 2), lane 1 A Z2Z2 (A of lane 2), lane 2 (2H)^2
    fdpp<kR2>(a, o2);                                    // lane 0: B
    fdpp<kR1>(b, o1);                                    // lane 1: A
    sel(P3, T.r0, a, b);
    sel(P3, T.r2, h2, P3);
    sel(Q3, T.r2, h2, o1);
    mul(o3, P3, Q3);                                     // (S2 | S1 | I)
    // lane 2: r = 2 (S2 - S1)
    fdpp<kL2>(s2, o3);                                   // lane 0's S2 at lane 2
    fdpp<kL1>(s1, o3);                                   // lane 1's S1 at lane 2
    fe26_sub<2>(rr, s2, s1);                             //                              m 3
    fe26_mul_int<2>(rr, rr);                             // r                            m 6
    // L4: lane 0 J = H I, lane 1 V = U1 I, lane 2 r^2 (H and I of lane 2)
    fdpp<kR2>(a, h);                                     // lane 0: H
    sel(P4, T.r0, a, o2);                                // (H | U1 | -)
    sel(P4, T.r2, rr, P4);                               // (H | U1 | r)
    fdpp<kR2>(a, o3);                                    // lane 0: I
    fdpp<kR1>(b, o3);                                    // lane 1: I
    sel(Q4, T.r0, a, b);
    sel(Q4, T.r2, rr, Q4);                               // (I | I | r)
    mul(o4, P4, Q4);                                     // (J | V | r^2)
    // lane 0: X3 = r^2 - J - 2V (r^2 of lane 2, V of lane 1), V - X3
    fdpp<kR2>(rv, o4);                                   // lane 0: r^2
    fdpp<kR1>(b, o4);                                    // lane 0: V
    fe26_sub<2>(X3, rv, o4);                             //                              m 3
    fe26_mul_int<2>(t, b);                               //                              m 2
    fe26_sub<3>(X3, X3, t);                              // X3                           m 6
    fe26_sub<7>(W, b, X3);                               // V - X3                       m 8
    // L5: lane 0 r (V - X3) (r of lane 2), lane 1 S1 J (J of lane 0), lane 2 Z1 Z2
    fdpp<kR2>(a, rr);                                    // lane 0: r
    sel(P5, T.r0, a, o3);                                // (r | S1 | -)
    sel(P5, T.r2, P.Zs, P5);                             // (r | S1 | Z1)
    fdpp<kL1>(b, o4);                                    // lane 1: J
    sel(Q5, T.r0, W, b);
    sel(Q5, T.r2, Q.Zs, Q5);                             // (V - X3 | J | Z2)
    mul(o5, P5, Q5);                                     // (r (V - X3) | S1 J | Z1 Z2)
    // L6 (lane 2): Z3 = 2 Z1 Z2 H
    mul(Z3, o5, h);
    fe26_mul_int<2>(Z3, Z3);                             //                              m 2
    // lane 0: Y3 = r (V - X3) - 2 S1 J
    fdpp<kR1>(t, o5);                                    // lane 0: S1 J
    fe26_mul_int<2>(t, t);                               //                              m 2
    fe26_sub<3>(Y3, o5, t);                              // Y3                           m 4
    TrioPt O;
    sel_dpp2<kL1, kL2>(O.S1, T.r0, X3, T.r1, Y3);      // (X3 | Y3 | Y3) from lane 0
    fdpp<kL2>(O.Xs, X3);                                 // lane 2 <- X3 of lane 0
    fe26_copy(O.Zs, Z3);
    O.inf = false;
    // exceptional cases (flags of lane 2, shared across the trio)
    const uint32_t zf = (fe26_is_zero(h) ? 1u : 0u) | (fe26_is_zero(rr) ? 2u : 0u);
    const uint32_t f = bdpp_from(zf, T, 2);
    const bool hz = (f & 1u) != 0u && !P.inf && !Q.inf;
    const bool rz = (f & 2u) != 0u;
    if (any(hz && rz)) {                                 // P == Q: double P on lane 2 (rare)
        Jac26 A, D;
        fe26_copy(A.X, P.Xs);
        fe26_copy(A.Y, P.S1);
        fe26_copy(A.Z, P.Zs);
        A.inf = P.inf;
        CurveK1x::dbl(D, A);
        TrioPt Dt;
        sel_dpp2<kR2, kR1>(Dt.S1, T.r2, D.Y, T.r0, D.X);  // lane 0 <- X, lane 1 <- Y of lane 2
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const uint32_t y = dpp<kR1>(D.Y.v[i]);
            Dt.S1.v[i] = T.r1 ? y : Dt.S1.v[i];
        }
        F26_SETM(Dt.S1, 10);
        fe26_copy(Dt.Xs, D.X);
        fe26_copy(Dt.Zs, D.Z);
        Dt.inf = false;
        trio_cmov(O, Dt, hz && rz);
    }
    if (hz && !rz) O.inf = true;                         // P == -Q
    trio_cmov(O, Q, P.inf);                              // (element-wise: no struct select through memory)
    trio_cmov(O, P, !P.inf && Q.inf);
    R = O;
}

}  // namespace bcosgpu
