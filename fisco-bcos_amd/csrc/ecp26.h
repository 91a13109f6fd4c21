// ecp26.h -- SM2 point arithmetic (a = -3) over fp26 (fp26.h, Montgomery R = 2^286): Jacobian
// coordinates, the formulas of ec.h's Curve<FieldP2, true> rearranged for fp26's magnitude contracts
// (mul/sqr inputs <= 15), so that no coordinate needs a weak normalisation (a serial nine-limb carry
// chain: ten of them per Booth window were ~5 % of the SM2 throughput kernel's instructions):
//   dbl  (dbl-2001-b, Z3 = 2 Y Z) : X <= 12, Y, Z <= 15                 -> (11, 11, 2)   4M + 4S
//   madd (madd-2007-bl, r/2)     : X, Y <= 11, Z <= 15; Q <= 11       -> (11, 11, 2)   8M + 3S
//   add  (add-2007-bl)           : X <= 12, Y, Z <= 15 (both)          -> (12, 15, 15)
// (madd / add outputs at their largest in the exceptional branches: the doubling, or an input passed
// through.)  Complete in the same cases as ec.h.  Checked by the FE26_CHECK host build
// (tests/cpp/fp26_test.cpp).
#pragma once
#include "fp26.h"

namespace bcosgpu {

struct JacP26 {
    fp26 X, Y, Z;
    bool inf;
};
struct AffP26 {
    fp26 x, y;
};

struct CurveSM2x {
    F26_HD static void set_inf(JacP26& R) {
        fp26_zero(R.X);
        fp26_set(R.Y, p26::ONE_R);
        fp26_zero(R.Z);
        R.inf = true;
    }
    F26_HD static void from_aff(JacP26& R, const AffP26& A) {
        fp26_copy(R.X, A.x);
        fp26_copy(R.Y, A.y);
        fp26_set(R.Z, p26::ONE_R);
        R.inf = false;
    }
    F26_HD static void cmov(JacP26& R, const JacP26& A, bool c) {
        fp26_cmov(R.X, A.X, c);
        fp26_cmov(R.Y, A.Y, c);
        fp26_cmov(R.Z, A.Z, c);
        R.inf = c ? A.inf : R.inf;
    }

    F26_HD static void dbl(JacP26& R, const JacP26& P) {
        fp26 delta, gamma, beta, t, u, alpha, a2, X3, Y3, Z3, g2;
        fp26_sqr(delta, P.Z);
        fp26_sqr(gamma, P.Y);
        fp26_mul(beta, P.X, gamma);
        fp26_sub<2>(t, P.X, delta);      // X - delta                  m X + 3
        fp26_add(u, P.X, delta);         // X + delta                  m X + 1
        fp26_mul(alpha, t, u);
        fp26_mul_int<3>(alpha, alpha);   // alpha = 3 (X - d)(X + d)   m 3
        fp26_sqr(a2, alpha);
        fp26_mul_int<8>(t, beta);        // 8 beta                     m 8
        fp26_sub<9>(X3, a2, t);          // X3 = alpha^2 - 8 beta      m 11
        fp26_mul(Z3, P.Y, P.Z);
        fp26_mul_int<2>(Z3, Z3);         // Z3 = 2 Y Z = (Y + Z)^2 - gamma - delta   m 2
        fp26_mul_int<12>(t, beta);       // 12 beta                    m 12
        fp26_sub<2>(t, t, a2);           // 4 beta - X3 = 12 beta - alpha^2   m 15
        fp26_mul(Y3, alpha, t);
        fp26_sqr(g2, gamma);
        fp26_mul_int<8>(g2, g2);         // 8 gamma^2                  m 8
        fp26_sub<9>(Y3, Y3, g2);         // Y3 = alpha (4 beta - X3) - 8 gamma^2   m 11
        fp26_copy(R.X, X3);
        fp26_copy(R.Y, Y3);
        fp26_copy(R.Z, Z3);
        R.inf = P.inf;
    }

    // R = P + Q, Q affine (never infinity)
    F26_HD static void madd(JacP26& R, const JacP26& P, const AffP26& Q) {
        fp26 Z1Z1, U2, S2, H, HH, I, J, rr, V, X3, Y3, Z3, t;
        fp26_sqr(Z1Z1, P.Z);
        fp26_mul(U2, Q.x, Z1Z1);
        fp26_mul(S2, Q.y, P.Z);
        fp26_mul(S2, S2, Z1Z1);
        fp26_sub<12>(H, U2, P.X);        // H = U2 - X1                m 14
        fp26_sqr(HH, H);
        fp26_mul_int<4>(I, HH);          // I = 4 HH                   m 4
        fp26_mul(J, H, I);
        fp26_sub<12>(rr, S2, P.Y);       // rr = S2 - Y1 = r / 2       m 14
        fp26_mul(V, P.X, I);
        fp26_sqr(X3, rr);
        fp26_mul_int<4>(X3, X3);         // r^2                        m 4
        fp26_sub<2>(X3, X3, J);          //                            m 7
        fp26_mul_int<2>(t, V);           //                            m 2
        fp26_sub<3>(X3, X3, t);          // X3 = r^2 - J - 2V          m 11
        fp26_sub<12>(t, V, X3);          // V - X3                     m 14
        fp26_mul(Y3, rr, t);
        fp26_mul(t, P.Y, J);
        fp26_sub<2>(Y3, Y3, t);          //                            m 4
        fp26_mul_int<2>(Y3, Y3);         // Y3 = r (V - X3) - 2 Y1 J   m 8
        fp26_mul(Z3, P.Z, H);
        fp26_mul_int<2>(Z3, Z3);         // Z3 = 2 Z1 H                m 2
        const bool hz = fp26_is_zero(H) && !P.inf;
        const bool rz = fp26_is_zero(rr);
        JacP26 D;
        if (hz && rz) dbl(D, P);         // P == Q (rare)
        const bool pinf = P.inf;
        fp26_copy(R.X, X3);
        fp26_copy(R.Y, Y3);
        fp26_copy(R.Z, Z3);
        R.inf = false;
        if (hz) {
            if (rz) cmov(R, D, true);
            else R.inf = true;
        }
        if (pinf) {
            fp26_copy(R.X, Q.x);
            fp26_copy(R.Y, Q.y);
            fp26_set(R.Z, p26::ONE_R);
            R.inf = false;
        }
    }

    // R = P + Q (Jacobian)
    F26_HD static void add(JacP26& R, const JacP26& P, const JacP26& Q) {
        fp26 Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, X3, Y3, Z3, t;
        fp26_sqr(Z1Z1, P.Z);
        fp26_sqr(Z2Z2, Q.Z);
        fp26_mul(U1, P.X, Z2Z2);
        fp26_mul(U2, Q.X, Z1Z1);
        fp26_mul(S1, P.Y, Q.Z);
        fp26_mul(S1, S1, Z2Z2);
        fp26_mul(S2, Q.Y, P.Z);
        fp26_mul(S2, S2, Z1Z1);
        fp26_sub<2>(H, U2, U1);          // m 4
        fp26_mul_int<2>(t, H);           // m 8
        fp26_sqr(I, t);                  // I = (2H)^2
        fp26_mul(J, H, I);
        fp26_sub<2>(rr, S2, S1);         // m 4
        fp26_mul_int<2>(rr, rr);         // r = 2 (S2 - S1)            m 8
        fp26_mul(V, U1, I);
        fp26_sqr(X3, rr);
        fp26_sub<2>(X3, X3, J);          // m 4
        fp26_mul_int<2>(t, V);           // m 2
        fp26_sub<3>(X3, X3, t);          // X3 = r^2 - J - 2V          m 8
        fp26_sub<9>(t, V, X3);           // m 11
        fp26_mul(Y3, rr, t);
        fp26_mul(t, S1, J);
        fp26_mul_int<2>(t, t);           // m 2
        fp26_sub<3>(Y3, Y3, t);          // Y3 = r (V - X3) - 2 S1 J   m 5
        fp26_mul(Z3, P.Z, Q.Z);
        fp26_mul(Z3, Z3, H);
        fp26_mul_int<2>(Z3, Z3);         // Z3 = 2 Z1 Z2 H             m 2
        const bool hz = fp26_is_zero(H) && !P.inf && !Q.inf;
        const bool rz = fp26_is_zero(rr);
        JacP26 D;
        if (hz && rz) dbl(D, P);
        JacP26 O;  // assembled apart from R, which may alias P or Q
        fp26_copy(O.X, X3);
        fp26_copy(O.Y, Y3);
        fp26_copy(O.Z, Z3);
        O.inf = false;
        if (hz) {
            if (rz) cmov(O, D, true);
            else O.inf = true;
        }
        if (P.inf) cmov(O, Q, true);
        else if (Q.inf) cmov(O, P, true);
        R = O;
    }
};

}  // namespace bcosgpu
