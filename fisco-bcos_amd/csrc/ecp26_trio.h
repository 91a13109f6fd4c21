// ecp26_trio.h -- SM2 (a = -3) doubling and mixed addition over fp26 split across a lane trio, as
// ec26_trio.h does for secp256k1 (same lanes, same DPP routing and role selects, same fences).  The
// formulas and magnitudes are CurveSM2x's (ecp26.h):
//
//   dbl (4 levels): L1  delta = Z^2       | gamma = Y^2       | Y Z
//                   L2  (X - d)(X + d)    | beta = X gamma    | gamma^2     (lane 2 fetches gamma)
//                   L3  alpha^2           | --                | --          (alpha = 3 (X - d)(X + d))
//                   L4  alpha (4 beta - X3) on lane 0, which fetches beta and gamma^2
//                   X3 = alpha^2 - 8 beta, Y3 = alpha (4 beta - X3) - 8 gamma^2, Z3 = 2 Y Z
//   madd (5 levels): the secp256k1 split (Z^2 | y2 Z | Z^2 -> U2 | S2 | U2 -> H^2 | rr^2 | Z H ->
//                   J | - | V -> rr (V - X3) | Y J), with CurveSM2x's weak normalisations
//
// a = -3 makes alpha^3 a degree-12 term, so the doubling above keeps four product levels (secp256k1's
// has three) -- unless delta = Z^2 travels with the point: the SM2 trio kernel's chain uses
// trio_dbl_sm2_d / trio_madd_sm2_d below (three levels per doubling, four per addition).  A point
// lives in the trio as TrioPtP: P1 = (Z | Y | Y) and Q1 = (Z | Y | Z) (the first doubling level's
// operands), Xr = (X | X | -); inf on every lane.  dbl: X <= 5, Y, Z <= 8 ->
// (2, 2, 2); madd: X, Y <= 2, Z <= 8, Q <= 2 -> (2, 2, 2).
#pragma once
#include "ec26_trio.h"
#include "ecp26.h"

namespace bcosgpu {

namespace trio {
F26_HD void mul(fp26& r, const fp26& a, const fp26& b) {
    fp26_mul(r, a, b);
    dpp_fence(r);
}
F26_HD void sqr(fp26& r, const fp26& a) {
    fp26_sqr(r, a);
    dpp_fence(r);
}
}  // namespace trio

struct TrioPtP {
    fp26 P1, Q1, Xr;
    bool inf;
};

F26_HD void trio_from_aff_sm2(TrioPtP& P, const AffP26& Q, const TrioLane& T) {
    fp26 one;
    fp26_set(one, p26::ONE_R);
    trio::sel(P.P1, T.r0, one, Q.y);
    trio::sel(P.Q1, T.r1, Q.y, one);
    fp26_copy(P.Xr, Q.x);
    P.inf = false;
}
F26_HD void trio_set_inf_sm2(TrioPtP& P) {
    fp26_zero(P.P1);
    fp26_zero(P.Q1);
    fp26_zero(P.Xr);
    P.inf = true;
}
F26_HD void trio_cmov_sm2(TrioPtP& P, const TrioPtP& Q, bool c) {
    fp26_cmov(P.P1, Q.P1, c);
    fp26_cmov(P.Q1, Q.Q1, c);
    fp26_cmov(P.Xr, Q.Xr, c);
    P.inf = c ? Q.inf : P.inf;
}
// the full Jacobian point on every lane (X from lane 0's Xr, Y from lane 1's P1, Z from lane 2's Q1)
F26_HD void trio_to_jac_sm2(JacP26& J, const TrioPtP& P, const TrioLane& T) {
    using namespace trio;
    sel_dpp2<kL1, kL2>(J.X, T.r0, P.Xr, T.r1, P.Xr);
    sel_dpp2<kR1, kL1>(J.Y, T.r1, P.P1, T.r0, P.P1);
    sel_dpp2<kR1, kR2>(J.Z, T.r2, P.Q1, T.r1, P.Q1);
    J.inf = P.inf;
}

// next state from X3, Y3 on lane 0 and Z3 on lane 2
F26_HD void trio_state_sm2(TrioPtP& O, const fp26& X3, const fp26& Y3, const fp26& Z3, const TrioLane& T) {
    using namespace trio;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t z0 = dpp<kR2>(Z3.v[i]), y1 = dpp<kL1>(Y3.v[i]), y2 = dpp<kL2>(Y3.v[i]),
                       x1 = dpp<kL1>(X3.v[i]);
        O.P1.v[i] = T.r0 ? z0 : T.r1 ? y1 : y2;
        O.Q1.v[i] = T.r0 ? z0 : T.r1 ? y1 : Z3.v[i];
        O.Xr.v[i] = T.r0 ? X3.v[i] : x1;
    }
#ifdef FE26_CHECK
    {
        const int mz0 = mdpp<kR2>(Z3.m), my1 = mdpp<kL1>(Y3.m), my2 = mdpp<kL2>(Y3.m), mx1 = mdpp<kL1>(X3.m);
        O.P1.m = T.r0 ? mz0 : T.r1 ? my1 : my2;
        O.Q1.m = T.r0 ? mz0 : T.r1 ? my1 : Z3.m;
        O.Xr.m = T.r0 ? X3.m : mx1;
    }
#endif
}

// P <- 2P
F26_HD void trio_dbl_sm2(TrioPtP& P, const TrioLane& T) {
    using namespace trio;
    fp26 o1, t, u, g, P2, Q2, o2, al, o3, be, g2, b8, X3, t4, Y3p, Y3, Z3;
    mul(o1, P.P1, P.Q1);                 // (delta | gamma | Y Z)
    fp26_sub<2>(t, P.Xr, o1);            // lane 0: X - delta          m X + 3
    fp26_add(u, P.Xr, o1);               // lane 0: X + delta          m X + 1
    fdpp<kL1>(g, o1);                    // lane 2: gamma of lane 1
    sel(P2, T.r0, t, P.Xr);
    sel(P2, T.r2, g, P2);                // (X - d | X | gamma)
    sel(Q2, T.r0, u, o1);
    sel(Q2, T.r2, g, Q2);                // (X + d | gamma | gamma)
    mul(o2, P2, Q2);                     // (alpha / 3 | beta | gamma^2)
    fp26_mul_int<3>(al, o2);             // lane 0: alpha              m 3
    sqr(o3, al);                         // lane 0: alpha^2
    fdpp<kR1>(be, o2);                   // lane 0: beta
    fdpp<kR2>(g2, o2);                   // lane 0: gamma^2
    fp26_mul_int<8>(b8, be);             //                            m 8
    fp26_sub<9>(X3, o3, b8);             //                            m 11
    fp26_normalize_weak(X3);             // X3 = alpha^2 - 8 beta      m 2
    fp26_mul_int<4>(t4, be);             //                            m 4
    fp26_sub<3>(t4, t4, X3);             // 4 beta - X3                m 8
    mul(Y3p, al, t4);
    fp26_mul_int<8>(g2, g2);             //                            m 8
    fp26_sub<9>(Y3, Y3p, g2);            //                            m 11
    fp26_normalize_weak(Y3);             // Y3                         m 2
    fp26_mul_int<2>(Z3, o1);             // lane 2: Z3 = 2 Y Z         m 2
    trio_state_sm2(P, X3, Y3, Z3, T);
}

// ---- the delta-carrying chain (the SM2 trio kernel's window): the point travels with D = delta = Z^2
// on lane 0, so a doubling needs no level for delta and takes THREE product levels:
//   L1  alpha / 3 = (X - D)(X + D) | gamma = Y^2     | Y Z
//   L2  alpha^2                    | beta = X gamma  | D' = (2 Y Z)^2  (the next delta = Z3^2)
//   L3  alpha (4 beta - X3)        | gamma^2         | --              (X3 = alpha^2 - 8 beta on lane 0)
// CurveSM2x::dbl's products, with no weak normalisation: fp26_mul takes magnitudes up to 15, so X3 and Y3
// go on unnormalised (each normalisation was a serial nine-limb carry chain on the critical path) and
// 4 beta - X3 is formed as 12 beta - alpha^2.  Magnitudes: X <= 12, Y, Z <= 15, D m 1 -> (11, 11, 2), D' m 1.
F26_HD void trio_dbl_sm2_d(TrioPtP& P, fp26& D, const TrioLane& T) {
    using namespace trio;
    fp26 t, u, A1, B1, o1, al, Z3, A2, B2, o2, be, b8, X3, t4, A3, B3, o3, g2, Y3, Dn;
    fp26_sub<2>(t, P.Xr, D);             // lane 0: X - delta          m X + 3
    fp26_add(u, P.Xr, D);                // lane 0: X + delta          m X + 1
    sel(A1, T.r0, t, P.P1);              // (X - d | Y | Y)
    sel(B1, T.r0, u, P.Q1);              // (X + d | Y | Z)
    mul(o1, A1, B1);                     // (alpha / 3 | gamma | Y Z)
    fp26_mul_int<3>(al, o1);             // lane 0: alpha              m 3
    fp26_mul_int<2>(Z3, o1);             // lane 2: Z3 = 2 Y Z         m 2
    sel(A2, T.r1, P.Xr, Z3);
    sel(A2, T.r0, al, A2);               // (alpha | X | Z3)
    sel(B2, T.r1, o1, Z3);
    sel(B2, T.r0, al, B2);               // (alpha | gamma | Z3)
    mul(o2, A2, B2);                     // (alpha^2 | beta | Z3^2)
    fdpp<kR1>(be, o2);                   // lane 0: beta
    fp26_mul_int<8>(b8, be);             //                            m 8
    fp26_sub<9>(X3, o2, b8);             // X3 = alpha^2 - 8 beta      m 11
    fp26_mul_int<12>(t4, be);            //                            m 12
    fp26_sub<2>(t4, t4, o2);             // 4 beta - X3 = 12 beta - alpha^2   m 15
    sel(A3, T.r0, al, o1);               // (alpha | gamma | -)
    sel(B3, T.r0, t4, o1);               // (4 beta - X3 | gamma | -)
    mul(o3, A3, B3);                     // (alpha (4 beta - X3) | gamma^2 | -)
    fdpp<kR1>(g2, o3);                   // lane 0: gamma^2
    fp26_mul_int<8>(g2, g2);             //                            m 8
    fp26_sub<9>(Y3, o3, g2);             // Y3                         m 11
    fdpp<kR2>(Dn, o2);                   // lane 0: Z3^2 of lane 2
    trio_state_sm2(P, X3, Y3, Z3, T);
    fp26_copy(D, Dn);
}

// R <- P + Q, Q affine, given D = Z1^2 on lane 0 (trio_dbl_sm2_d): CurveSM2x::madd in 4 product levels,
// without the P = +-Q tests (the t P chain's additions), returning the sum's D = Z3^2 on lane 0 from
// the last level's idle lane 2; P = infinity gives Q (D = 1).  No weak normalisations (fp26_mul takes
// m <= 15): X, Y <= 11, Z <= 15, D m 1, Q <= 2 -> (11, 8, 2), D m 1.
//   L1  U2 = x2 D        | T = y2 Z        | --
//   L2  HH = H^2         | S2 = T D        | Z H          (H = U2 - X on lane 0)
//   L3  J = H I          | rr^2            | V = X I      (I = 4 HH, rr = S2 - Y on lane 1)
//   L4  rr (V - X3)      | Y J             | Z3^2         (X3 = 4 rr^2 - J - 2V on lane 0, Z3 = 2 Z H)
F26_HD void trio_madd_sm2_d(TrioPtP& R, fp26& Dout, const TrioPtP& P, const fp26& D, const AffP26& Q,
                            const TrioLane& T) {
    using namespace trio;
    fp26 a, b, A1, B1, o1, h, A2, B2, o2, I, rr, A3, B3, o3, R2, V, X3, t, W, Z3, A4, B4, o4, Y3, Dn;
    fdpp<kR1>(b, P.Q1);                  // lane 1: Z of lane 2
    sel(A1, T.r1, Q.y, Q.x);             // (x2 | y2 | x2)
    sel(B1, T.r0, D, b);                 // (D | Z | -)
    mul(o1, A1, B1);                     // (U2 | T | -)
    fp26_sub<12>(h, o1, P.Xr);           // lane 0: H = U2 - X         m 14
    sel(A2, T.r1, o1, P.Q1);
    sel(A2, T.r0, h, A2);                // (H | T | Z)
    fdpp<kL1>(a, D);                     // lane 1: D of lane 0
    fdpp<kL2>(b, h);                     // lane 2: H of lane 0
    sel(B2, T.r1, a, b);
    sel(B2, T.r0, h, B2);                // (H | D | H)
    mul(o2, A2, B2);                     // (HH | S2 | Z H)
    fp26_mul_int<4>(I, o2);              // lane 0: I = 4 HH           m 4
    fp26_sub<12>(rr, o2, P.P1);          // lane 1: rr = S2 - Y        m 14
    fp26_mul_int<2>(Z3, o2);             // lane 2: Z3 = 2 Z H         m 2
    fdpp<kL1>(a, P.Xr);                  // lane 2: X of lane 1
    sel(A3, T.r1, rr, a);
    sel(A3, T.r0, h, A3);                // (H | rr | X)
    fdpp<kL2>(b, I);                     // lane 2: I of lane 0
    sel(B3, T.r1, rr, b);
    sel(B3, T.r0, I, B3);                // (I | rr | I)
    mul(o3, A3, B3);                     // (J | rr^2 | V)
    fdpp<kR1>(R2, o3);
    fp26_mul_int<4>(R2, R2);             // lane 0: r^2 = 4 rr^2       m 4
    fdpp<kR2>(V, o3);                    // lane 0: V
    fp26_sub<2>(X3, R2, o3);             //                            m 7
    fp26_mul_int<2>(t, V);               //                            m 2
    fp26_sub<3>(X3, X3, t);              // X3 = r^2 - J - 2V          m 11
    fp26_sub<12>(W, V, X3);              // V - X3                     m 14
    fdpp<kR1>(a, rr);                    // lane 0: rr of lane 1       m 14
    sel(A4, T.r1, P.P1, Z3);
    sel(A4, T.r0, a, A4);                // (rr | Y | Z3)
    fdpp<kL1>(b, o3);                    // lane 1: J of lane 0
    sel(B4, T.r1, b, Z3);
    sel(B4, T.r0, W, B4);                // (V - X3 | J | Z3)
    mul(o4, A4, B4);                     // (rr (V - X3) | Y J | Z3^2)
    fdpp<kR1>(t, o4);
    fp26_sub<2>(Y3, o4, t);              //                            m 4
    fp26_mul_int<2>(Y3, Y3);             // Y3 = r (V - X3) - 2 Y J    m 8
    fdpp<kR2>(Dn, o4);                   // lane 0: Z3^2 of lane 2
    TrioPtP O;
    trio_state_sm2(O, X3, Y3, Z3, T);
    O.inf = false;
    if (P.inf) {
        trio_from_aff_sm2(O, Q, T);
        fp26_set(Dn, p26::ONE_R);
    }
    R = O;
    fp26_copy(Dout, Dn);
}

// a Jacobian table entry with its Z powers (the SM2 trio kernel's chain adds these while the affine
// table is still being built): every element m 1
struct JacEntP26 {
    fp26 X, Y, Z, ZZ, ZZZ;
};

// R <- P + Q, Q a Jacobian table entry (never infinity), given D = Z1^2 on lane 0: CurveSM2x::add's
// point in 5 product levels, without the P = +-Q tests (as trio_madd_sm2_d), returning the sum's
// D = Z3^2 on lane 0; P = infinity gives Q (D = ZZ2).  No weak normalisations (fp26_mul takes m <= 15):
// X, Y, Z <= 15, D m 1 -> (11, 8, 2), D m 1.
//   L1  U2 = X2 D        | T = Y2 Z1       | U1 = X1 ZZ2
//   L2  Z1 Z2            | S2 = T D        | S1 = Y1 ZZZ2   (H = U2 - U1 on lane 0)
//   L3  HH = H^2         | rr^2            | Z1 Z2 H        (rr = S2 - S1 on lane 1)
//   L4  J = H I          | Z3^2            | V = U1 I       (I = 4 HH, Z3 = 2 Z1 Z2 H)
//   L5  rr (V - X3)      | S1 J            | --             (X3 = 4 rr^2 - J - 2V on lane 0)
F26_HD void trio_add_sm2_jd(TrioPtP& R, fp26& Dout, const TrioPtP& P, const fp26& D, const JacEntP26& Q,
                            const TrioLane& T) {
    using namespace trio;
    fp26 a, b, A1, B1, o1, h, A2, B2, o2, rr, A3, B3, o3, I, Z3, R2, A4, B4, o4, V, X3, t, W, A5, B5, o5, Y3, Dn;
    fdpp<kR1>(a, P.Q1);                  // lane 1: Z of lane 2
    fdpp<kL1>(b, P.Xr);                  // lane 2: X of lane 1
    sel(A1, T.r1, Q.Y, Q.X);
    sel(A1, T.r2, b, A1);                // (X2 | Y2 | X1)
    sel(B1, T.r1, a, Q.ZZ);
    sel(B1, T.r0, D, B1);                // (D | Z1 | ZZ2)
    mul(o1, A1, B1);                     // (U2 | T | U1)
    fdpp<kR2>(a, o1);                    // lane 0: U1 of lane 2
    fp26_sub<2>(h, o1, a);               // lane 0: H = U2 - U1        m 4
    fdpp<kL1>(b, D);                     // lane 1: D of lane 0
    sel(B2, T.r1, b, Q.ZZZ);
    sel(B2, T.r0, Q.Z, B2);              // (Z2 | D | ZZZ2)
    sel(A2, T.r1, o1, P.P1);             // (Z1 | T | Y1)
    mul(o2, A2, B2);                     // (Z1 Z2 | S2 | S1)
    fdpp<kR1>(a, o2);                    // lane 1: S1 of lane 2
    fp26_sub<2>(rr, o2, a);              // lane 1: rr = S2 - S1       m 4
    fdpp<kL2>(a, o2);                    // lane 2: Z1 Z2 of lane 0
    fdpp<kL2>(b, h);                     // lane 2: H of lane 0
    sel(A3, T.r1, rr, a);
    sel(A3, T.r0, h, A3);                // (H | rr | Z1 Z2)
    sel(B3, T.r1, rr, b);
    sel(B3, T.r0, h, B3);                // (H | rr | H)
    mul(o3, A3, B3);                     // (HH | rr^2 | Z1 Z2 H)
    fp26_mul_int<4>(I, o3);              // lane 0: I = 4 HH           m 4
    fp26_mul_int<2>(Z3, o3);             // lane 2: Z3 = 2 Z1 Z2 H     m 2
    fdpp<kR1>(R2, o3);
    fp26_mul_int<4>(R2, R2);             // lane 0: r^2 = 4 rr^2       m 4
    fdpp<kR1>(a, Z3);                    // lane 1: Z3 of lane 2
    fdpp<kL2>(b, I);                     // lane 2: I of lane 0
    sel(A4, T.r1, a, o1);
    sel(A4, T.r0, h, A4);                // (H | Z3 | U1)
    sel(B4, T.r1, a, b);
    sel(B4, T.r0, I, B4);                // (I | Z3 | I)
    mul(o4, A4, B4);                     // (J | Z3^2 | V)
    fdpp<kR2>(V, o4);                    // lane 0: V
    fp26_sub<2>(X3, R2, o4);             //                            m 7
    fp26_mul_int<2>(t, V);               //                            m 2
    fp26_sub<3>(X3, X3, t);              // X3 = r^2 - J - 2V          m 11
    fp26_sub<12>(W, V, X3);              // V - X3                     m 14
    fdpp<kR1>(a, rr);                    // lane 0: rr of lane 1       m 4
    fdpp<kR1>(b, o2);                    // lane 1: S1 of lane 2
    sel(A5, T.r0, a, b);                 // (rr | S1 | -)
    fdpp<kL1>(b, o4);                    // lane 1: J of lane 0
    sel(B5, T.r0, W, b);                 // (V - X3 | J | -)
    mul(o5, A5, B5);                     // (rr (V - X3) | S1 J | -)
    fdpp<kR1>(t, o5);
    fp26_sub<2>(Y3, o5, t);              //                            m 4
    fp26_mul_int<2>(Y3, Y3);             // Y3 = r (V - X3) - 2 S1 J   m 8
    fdpp<kR1>(Dn, o4);                   // lane 0: Z3^2 of lane 1
    TrioPtP O;
    trio_state_sm2(O, X3, Y3, Z3, T);
    O.inf = false;
    if (P.inf) {
        trio::sel(O.P1, T.r0, Q.Z, Q.Y);
        trio::sel(O.Q1, T.r1, Q.Y, Q.Z);
        fp26_copy(O.Xr, Q.X);
        fp26_copy(Dn, Q.ZZ);
    }
    R = O;
    fp26_copy(Dout, Dn);
}

// R <- P + Q (Q affine, never infinity); exceptional cases as CurveSM2x::madd, EXC = false drops the
// P = +-Q tests for callers that exclude them (see the SM2 trio kernel in ecc_pair.hip)
template <bool EXC = true>
F26_HD void trio_madd_sm2(TrioPtP& R, const TrioPtP& P, const AffP26& Q, const TrioLane& T) {
    using namespace trio;
    fp26 q1r, Zb, xl1, Xl, P1, o1, P2, Q2, o2, h, P3, o3, HHx, I, P4, o4, R2, V, X3, t, W, rr, P5, Q5, J1, o5, Y3, Z3;
    fdpp<kR1>(q1r, P.Q1);
    sel(Zb, T.r1, q1r, P.P1);
    sel(Zb, T.r2, P.Q1, Zb);             // Z on every lane            m <= 8
    fdpp<kL1>(xl1, P.Xr);
    sel(Xl, T.r2, xl1, P.Xr);
    sel(Xl, T.r1, P.P1, Xl);             // (X | Y | X)                m <= 2
    sel(P1, T.r1, Q.y, Zb);
    mul(o1, P1, Zb);                     // (Z1Z1 | y2 Z | Z1Z1)
    sel(P2, T.r1, o1, Q.x);
    fdpp<kR1>(Q2, o1);
    sel(Q2, T.r1, Q2, o1);
    mul(o2, P2, Q2);                     // (U2 | S2 | U2)
    fp26_sub<3>(h, o2, Xl);              // (H | rr | H)               m 5
    sel(P3, T.r2, Zb, h);
    mul(o3, P3, h);                      // (HH | rr^2 | Z H)
    fdpp<kL2>(HHx, o3);
    sel(HHx, T.r2, HHx, o3);
    fp26_mul_int<4>(I, HHx);             // I = 4 HH                   m 4
    sel(P4, T.r2, Xl, h);
    mul(o4, P4, I);                      // (J | - | V)
    fdpp<kR1>(R2, o3);
    fp26_mul_int<4>(R2, R2);             // lane 0: r^2 = 4 rr^2       m 4
    fdpp<kR2>(V, o4);                    // lane 0: V
    fp26_sub<2>(X3, R2, o4);             //                            m 7
    fp26_mul_int<2>(t, V);               //                            m 2
    fp26_sub<3>(X3, X3, t);              //                            m 11
    fp26_normalize_weak(X3);             // X3 = r^2 - J - 2V          m 2
    fp26_sub<3>(W, V, X3);               // V - X3                     m 5
    fdpp<kR1>(rr, h);                    // lane 0: rr                 m 5
    sel(P5, T.r0, rr, P.P1);             // lane 0: rr, lane 1: Y
    fdpp<kL1>(J1, o4);
    sel(Q5, T.r0, W, J1);                // lane 0: V - X3, lane 1: J
    mul(o5, P5, Q5);                     // (rr (V - X3) | Y J | -)
    fdpp<kR1>(t, o5);
    fp26_sub<2>(Y3, o5, t);              //                            m 4
    fp26_mul_int<2>(Y3, Y3);             //                            m 8
    fp26_normalize_weak(Y3);             // Y3 = r (V - X3) - 2 Y J    m 2
    fp26_mul_int<2>(Z3, o3);             // lane 2: Z3 = 2 Z H         m 2
    TrioPtP O;
    trio_state_sm2(O, X3, Y3, Z3, T);
    O.inf = false;
    if constexpr (EXC) {
        const uint32_t zf = fp26_is_zero(h) ? 1u : 0u;
        const bool hz = bdpp_from(zf, T, 0) != 0u && !P.inf;
        const bool rz = bdpp_from(zf, T, 1) != 0u;
        if (any(hz && rz)) {  // P == Q: double on lane 2, which holds X (Xl), Y (P1) and Z (Q1)
            JacP26 A, D;
            fp26_copy(A.X, Xl);
            fp26_copy(A.Y, P.P1);
            fp26_copy(A.Z, P.Q1);
            A.inf = P.inf;
            CurveSM2x::dbl(D, A);
            fp26_normalize_weak(D.X);  // the chain's magnitudes (2, 2, 2)
            fp26_normalize_weak(D.Y);
            // D on lane 2 -> X3, Y3 on lane 0 and Z3 on lane 2, then the usual state
            fp26 dx, dy;
            fdpp<kR2>(dx, D.X);
            fdpp<kR2>(dy, D.Y);
            TrioPtP Dt;
            trio_state_sm2(Dt, dx, dy, D.Z, T);
            Dt.inf = false;
            trio_cmov_sm2(O, Dt, hz && rz);
        }
        if (hz && !rz) O.inf = true;  // P == -Q
    }
    if (P.inf) trio_from_aff_sm2(O, Q, T);
    R = O;
}

}  // namespace bcosgpu
