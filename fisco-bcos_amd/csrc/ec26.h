// ec26.h -- secp256k1 point arithmetic over the 10 x 26-bit field (fe26.h): Jacobian coordinates,
// one point per lane, the same formulas as ec.h's Curve<FieldK1, false> (dbl-2009-l with D = 4XB,
// madd-2007-bl, add-2007-bl, complete in the same cases) rearranged so that every intermediate stays
// within fe26's magnitude contracts.  The magnitudes each routine accepts and returns are part of its
// interface (checked at run time by the FE26_CHECK host build, tests/cpp/fe26_test.cpp):
//   dbl  : X, Y, Z <= 16                 -> (10, 10, 2)
//   madd : X, Y <= 10, Z <= 16; Q <= 2   -> (9, 6, 2)
//   add  : X, Y, Z <= 16 (both)          -> (6, 4, 2)
// so any sequence of doublings and additions keeps its inputs legal without normalising.
#pragma once
#include "fe26.h"

namespace bcosgpu {

struct Jac26 {
    fe26 X, Y, Z;
    bool inf;
};
struct Aff26 {
    fe26 x, y;
};

struct CurveK1x {
    F26_HD static void set_inf(Jac26& R) {
        fe26_zero(R.X);
        fe26_one(R.Y);
        fe26_zero(R.Z);
        R.inf = true;
    }
    F26_HD static void from_aff(Jac26& R, const Aff26& A) {
        fe26_copy(R.X, A.x);
        fe26_copy(R.Y, A.y);
        fe26_one(R.Z);
        R.inf = false;
    }
    F26_HD static void cmov(Jac26& R, const Jac26& A, bool c) {
        fe26_cmov(R.X, A.X, c);
        fe26_cmov(R.Y, A.Y, c);
        fe26_cmov(R.Z, A.Z, c);
        R.inf = c ? A.inf : R.inf;
    }

    F26_HD static void dbl(Jac26& R, const Jac26& P) {
        fe26 A, B, C, D, E, X3, Y3, Z3, t;
        fe26_sqr(A, P.X);
        fe26_sqr(B, P.Y);
        fe26_sqr(C, B);
        fe26_mul(D, P.X, B);
        fe26_mul_int<4>(D, D);      // D = 4 X B                  m 4
        fe26_mul_int<3>(E, A);      // E = 3 A                    m 3
        fe26_sqr(X3, E);
        fe26_mul_int<2>(t, D);      //                            m 8
        fe26_sub<9>(X3, X3, t);     // X3 = E^2 - 2D              m 10
        fe26_sub<11>(t, D, X3);     // D - X3                     m 15
        fe26_mul(Y3, E, t);
        fe26_mul_int<8>(C, C);      //                            m 8
        fe26_sub<9>(Y3, Y3, C);     // Y3 = E (D - X3) - 8C       m 10
        fe26_mul(Z3, P.Y, P.Z);
        fe26_mul_int<2>(Z3, Z3);    // Z3 = 2 Y Z                 m 2
        fe26_copy(R.X, X3);
        fe26_copy(R.Y, Y3);
        fe26_copy(R.Z, Z3);
        R.inf = P.inf;
    }

    // R = P + Q, Q affine (never infinity); r = 2 rr is carried as rr so r^2 = 4 rr^2 stays in range
    F26_HD static void madd(Jac26& R, const Jac26& P, const Aff26& Q) {
        fe26 Z1Z1, U2, S2, H, HH, I, J, rr, V, X3, Y3, Z3, t;
        fe26_sqr(Z1Z1, P.Z);
        fe26_mul(U2, Q.x, Z1Z1);
        fe26_mul(S2, Q.y, P.Z);
        fe26_mul(S2, S2, Z1Z1);
        fe26_sub<11>(H, U2, P.X);   // H = U2 - X1                m 12
        fe26_sqr(HH, H);
        fe26_mul_int<4>(I, HH);     // I = 4 HH                   m 4
        fe26_mul(J, H, I);
        fe26_sub<11>(rr, S2, P.Y);  // rr = S2 - Y1 = r / 2       m 12
        fe26_mul(V, P.X, I);
        fe26_sqr(X3, rr);
        fe26_mul_int<4>(X3, X3);    // r^2                        m 4
        fe26_sub<2>(X3, X3, J);     //                            m 6
        fe26_mul_int<2>(t, V);      //                            m 2
        fe26_sub<3>(X3, X3, t);     // X3 = r^2 - J - 2V          m 9
        fe26_sub<10>(t, V, X3);     // V - X3                     m 11
        fe26_mul(Y3, rr, t);
        fe26_mul(t, P.Y, J);
        fe26_sub<2>(Y3, Y3, t);     //                            m 3
        fe26_mul_int<2>(Y3, Y3);    // Y3 = r (V - X3) - 2 Y1 J   m 6
        fe26_mul(Z3, P.Z, H);
        fe26_mul_int<2>(Z3, Z3);    // Z3 = (Z1 + H)^2 - Z1Z1 - HH = 2 Z1 H   m 2
        const bool hz = fe26_is_zero(H) && !P.inf;
        const bool rz = fe26_is_zero(rr);
        Jac26 D;
        if (hz && rz) dbl(D, P);    // P == Q (rare)
        const bool pinf = P.inf;
        fe26_copy(R.X, X3);
        fe26_copy(R.Y, Y3);
        fe26_copy(R.Z, Z3);
        R.inf = false;
        if (hz) {
            if (rz) cmov(R, D, true);
            else R.inf = true;      // P == -Q
        }
        if (pinf) {
            fe26_copy(R.X, Q.x);
            fe26_copy(R.Y, Q.y);
            fe26_one(R.Z);
            R.inf = false;
        }
    }

    // R = P + Q (Jacobian)
    F26_HD static void add(Jac26& R, const Jac26& P, const Jac26& Q) {
        fe26 Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, X3, Y3, Z3, t;
        fe26_sqr(Z1Z1, P.Z);
        fe26_sqr(Z2Z2, Q.Z);
        fe26_mul(U1, P.X, Z2Z2);
        fe26_mul(U2, Q.X, Z1Z1);
        fe26_mul(S1, P.Y, Q.Z);
        fe26_mul(S1, S1, Z2Z2);
        fe26_mul(S2, Q.Y, P.Z);
        fe26_mul(S2, S2, Z1Z1);
        fe26_sub<2>(H, U2, U1);     // m 3
        fe26_mul_int<2>(t, H);      // m 6
        fe26_sqr(I, t);             // I = (2H)^2
        fe26_mul(J, H, I);
        fe26_sub<2>(rr, S2, S1);    // m 3
        fe26_mul_int<2>(rr, rr);    // r = 2 (S2 - S1)            m 6
        fe26_mul(V, U1, I);
        fe26_sqr(X3, rr);
        fe26_sub<2>(X3, X3, J);     // m 3
        fe26_mul_int<2>(t, V);      // m 2
        fe26_sub<3>(X3, X3, t);     // X3 = r^2 - J - 2V          m 6
        fe26_sub<7>(t, V, X3);      // m 8
        fe26_mul(Y3, rr, t);
        fe26_mul(t, S1, J);
        fe26_mul_int<2>(t, t);      // m 2
        fe26_sub<3>(Y3, Y3, t);     // Y3 = r (V - X3) - 2 S1 J   m 4
        fe26_mul(Z3, P.Z, Q.Z);
        fe26_mul(Z3, Z3, H);
        fe26_mul_int<2>(Z3, Z3);    // Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H = 2 Z1 Z2 H   m 2
        const bool hz = fe26_is_zero(H) && !P.inf && !Q.inf;
        const bool rz = fe26_is_zero(rr);
        Jac26 D;
        if (hz && rz) dbl(D, P);
        Jac26 O;  // assembled apart from R, which may alias P or Q
        fe26_copy(O.X, X3);
        fe26_copy(O.Y, Y3);
        fe26_copy(O.Z, Z3);
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
