// ec.h -- short-Weierstrass point arithmetic for gfx950 (Jacobian coordinates, one point per lane).
//
// Curve<F, AM3>: F is the base field (FieldK1 for secp256k1, FieldP2 for SM2), AM3 selects the
// a = -3 doubling (SM2) over the a = 0 one (secp256k1).  Formulas (EFD names):
//   dbl  a=0 : dbl-2009-l, D = 4XB (3M + 4S)  dbl a=-3 : dbl-2001-b (3M + 5S)
//   madd     : madd-2007-bl (7M + 4S)      add      : add-2007-bl (11M + 5S)
// madd/add are complete: infinity operands, P == Q (-> doubling) and P == -Q (-> infinity) are
// handled, so results are exact for every input the reference accepts.  The rare branches are
// per-lane predicated; a wave skips them when no lane takes them.
#pragma once
#include "fe.h"
#include "modinv.h"

namespace bcosgpu {

struct Jac {
    fe X, Y, Z;
    bool inf;
};
struct Aff {
    fe x, y;
};

template <class F, bool AM3>
struct Curve {
    __device__ static __forceinline__ void set_inf(Jac& R) {
        fe_zero(R.X);
        F::set_one(R.Y);
        fe_zero(R.Z);
        R.inf = true;
    }
    __device__ static __forceinline__ void from_aff(Jac& R, const Aff& A) {
        fe_copy(R.X, A.x);
        fe_copy(R.Y, A.y);
        F::set_one(R.Z);
        R.inf = false;
    }
    __device__ static __forceinline__ void cmov(Jac& R, const Jac& A, bool c) {
        fe_cmov(R.X, A.X, c);
        fe_cmov(R.Y, A.Y, c);
        fe_cmov(R.Z, A.Z, c);
        R.inf = c ? A.inf : R.inf;
    }

    __device__ static __forceinline__ void dbl(Jac& R, const Jac& P) {
        fe X3, Y3, Z3;
        if (AM3) {
            fe delta, gamma, beta, alpha, t, u;
            F::sqr(delta, P.Z);
            F::sqr(gamma, P.Y);
            F::mul(beta, P.X, gamma);
            F::sub(t, P.X, delta);
            F::add(u, P.X, delta);
            F::mul(alpha, t, u);
            F::add(t, alpha, alpha);
            F::add(alpha, alpha, t);  // alpha = 3 (X - delta)(X + delta)
            F::add(t, P.Y, P.Z);
            F::sqr(Z3, t);
            F::sub(Z3, Z3, gamma);
            F::sub(Z3, Z3, delta);
            F::add(beta, beta, beta);
            F::add(beta, beta, beta);  // 4 beta
            F::sqr(X3, alpha);
            F::add(t, beta, beta);
            F::sub(X3, X3, t);  // alpha^2 - 8 beta
            F::sub(t, beta, X3);
            F::mul(Y3, alpha, t);
            F::sqr(u, gamma);
            F::add(u, u, u);
            F::add(u, u, u);
            F::add(u, u, u);  // 8 gamma^2
            F::sub(Y3, Y3, u);
        } else {
            // dbl-2009-l with D = 2((X + B)^2 - A - C) = 4 X B taken as a multiplication (3M + 4S):
            // the shifted passes replace ten of its fourteen field additions
            fe A, B, C, E, W, t;
            F::sqr(A, P.X);
            F::sqr(B, P.Y);
            F::sqr(C, B);
            F::mul(W, P.X, B);
            F::template shl<2>(W, W);  // D = 4 X B
            F::mul3(E, A);
            F::sqr(X3, E);
            F::template shl<1>(t, W);
            F::sub(X3, X3, t);         // E^2 - 2D
            F::sub(t, W, X3);
            F::mul(Y3, E, t);
            F::template shl<3>(C, C);
            F::sub(Y3, Y3, C);         // E (D - X3) - 8 C
            F::mul(Z3, P.Y, P.Z);
            F::template shl<1>(Z3, Z3);
        }
        fe_copy(R.X, X3);
        fe_copy(R.Y, Y3);
        fe_copy(R.Z, Z3);
        R.inf = P.inf;
    }

    // R = P + Q, Q affine (never infinity)
    __device__ static __forceinline__ void madd(Jac& R, const Jac& P, const Aff& Q) {
        fe Z1Z1, U2, S2, H, HH, I, J, rr, V, X3, Y3, Z3, t;
        F::sqr(Z1Z1, P.Z);
        F::mul(U2, Q.x, Z1Z1);
        F::mul(S2, Q.y, P.Z);
        F::mul(S2, S2, Z1Z1);
        F::sub(H, U2, P.X);
        F::sqr(HH, H);
        F::template shl<2>(I, HH);
        F::mul(J, H, I);
        F::sub(rr, S2, P.Y);
        F::template shl<1>(rr, rr);
        F::mul(V, P.X, I);
        F::sqr(X3, rr);
        F::sub(X3, X3, J);
        F::template shl<1>(t, V);
        F::sub(X3, X3, t);
        F::sub(t, V, X3);
        F::mul(Y3, rr, t);
        F::mul(t, P.Y, J);
        F::template shl<1>(t, t);
        F::sub(Y3, Y3, t);
        F::add(t, P.Z, H);
        F::sqr(Z3, t);
        F::sub(Z3, Z3, Z1Z1);
        F::sub(Z3, Z3, HH);
        const bool hz = F::is_zero(H) && !P.inf;
        const bool rz = F::is_zero(rr);
        Jac D;
        if (hz && rz) dbl(D, P);  // P == Q (rare)
        const bool pinf = P.inf;
        fe_copy(R.X, X3);
        fe_copy(R.Y, Y3);
        fe_copy(R.Z, Z3);
        R.inf = false;
        if (hz) {
            if (rz) cmov(R, D, true);
            else R.inf = true;  // P == -Q
        }
        if (pinf) {
            fe_copy(R.X, Q.x);
            fe_copy(R.Y, Q.y);
            F::set_one(R.Z);
            R.inf = false;
        }
    }

    // R = P + Q (Jacobian)
    __device__ static __forceinline__ void add(Jac& R, const Jac& P, const Jac& Q) {
        fe Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, X3, Y3, Z3, t;
        F::sqr(Z1Z1, P.Z);
        F::sqr(Z2Z2, Q.Z);
        F::mul(U1, P.X, Z2Z2);
        F::mul(U2, Q.X, Z1Z1);
        F::mul(S1, P.Y, Q.Z);
        F::mul(S1, S1, Z2Z2);
        F::mul(S2, Q.Y, P.Z);
        F::mul(S2, S2, Z1Z1);
        F::sub(H, U2, U1);
        F::add(t, H, H);
        F::sqr(I, t);
        F::mul(J, H, I);
        F::sub(rr, S2, S1);
        F::add(rr, rr, rr);
        F::mul(V, U1, I);
        F::sqr(X3, rr);
        F::sub(X3, X3, J);
        F::add(t, V, V);
        F::sub(X3, X3, t);
        F::sub(t, V, X3);
        F::mul(Y3, rr, t);
        F::mul(t, S1, J);
        F::add(t, t, t);
        F::sub(Y3, Y3, t);
        F::add(t, P.Z, Q.Z);
        F::sqr(Z3, t);
        F::sub(Z3, Z3, Z1Z1);
        F::sub(Z3, Z3, Z2Z2);
        F::mul(Z3, Z3, H);
        const bool hz = F::is_zero(H) && !P.inf && !Q.inf;
        const bool rz = F::is_zero(rr);
        Jac D;
        if (hz && rz) dbl(D, P);
        const bool pinf = P.inf, qinf = Q.inf;
        Jac Pc;
        if (qinf) Pc = P;
        fe_copy(R.X, X3);
        fe_copy(R.Y, Y3);
        fe_copy(R.Z, Z3);
        R.inf = false;
        if (hz) {
            if (rz) cmov(R, D, true);
            else R.inf = true;
        }
        if (pinf) cmov(R, Q, true);
        else if (qinf) cmov(R, Pc, true);
    }

    // affine coordinates in the field's internal form; returns false for infinity
    __device__ static __forceinline__ bool to_aff(Aff& A, const Jac& P) {
        fe zi, zi2, t;
        FieldInv<F>::inv(zi, P.Z);
        F::sqr(zi2, zi);
        F::mul(A.x, P.X, zi2);
        F::mul(t, zi2, zi);
        F::mul(A.y, P.Y, t);
        return !P.inf;
    }

    // y^2 == x^3 + a x + b for affine (x, y) in internal form
    __device__ static __forceinline__ bool on_curve(const Aff& A, const fe& b) {
        fe l, r, t;
        F::sqr(l, A.y);
        F::sqr(t, A.x);
        F::mul(r, t, A.x);
        if (AM3) {
            F::add(t, A.x, A.x);
            F::add(t, t, A.x);
            F::sub(r, r, t);
        }
        F::add(r, r, b);
        return F::eq(l, r);
    }
};

using CurveK1 = Curve<FieldK1, false>;
using CurveSM2 = Curve<FieldP2, true>;

}  // namespace bcosgpu
