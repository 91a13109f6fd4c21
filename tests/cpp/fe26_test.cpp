// fe26_test.cpp -- host build of fe26.h / ec26.h with FE26_CHECK: every magnitude contract and limb
// bound is asserted at run time while random and extreme operands go through the field operations and
// the point formulas.  Prints one line per case; tests/test_fe26.py recomputes each with Python
// integers (mod p, and affine secp256k1 arithmetic).
//   F <op> <a limbs> <b limbs> <r limbs>     field cases (value = sum limb_i 2^(26 i))
//   P <k hex> <X> <Y> <Z> <inf>              k*G by double-and-madd from an affine G
//   A <case> <X> <Y> <Z> <inf>               add/madd special cases (P+P, P-P, inf+Q, P+inf)
#define FE26_CHECK 1
#include "../../fisco-bcos_amd/csrc/ec26.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

using namespace bcosgpu;

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint32_t rnd() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return static_cast<uint32_t>(rng >> 11);
}

// a random element of magnitude m; mode 0 random limbs, 1 every limb at its bound, 2 zero limbs but one
static void rand_fe(fe26& a, int m, int mode) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t bound = static_cast<uint64_t>(m) << (i == 9 ? 22 : 26);
        uint64_t v;
        if (mode == 1) v = bound;
        else if (mode == 2) v = (i == static_cast<int>(rnd() % 10)) ? bound : 0;
        else v = (static_cast<uint64_t>(rnd()) << 20 ^ rnd()) % (bound + 1);
        a.v[i] = static_cast<uint32_t>(v);
    }
    a.m = m;
}

static void pr(const fe26& a) {
    for (int i = 0; i < 10; ++i) printf("%s%x", i ? "," : " ", a.v[i]);
}

static void field_case(const char* op, const fe26& a, const fe26& b, const fe26& r) {
    printf("F %s", op);
    pr(a);
    pr(b);
    pr(r);
    printf("\n");
}

static const uint32_t kGx[8] = {0x16f81798u, 0x59f2815bu, 0x2dce28d9u, 0x029bfcdbu,
                                0xce870b07u, 0x55a06295u, 0xf9dcbbacu, 0x79be667eu};
static const uint32_t kGy[8] = {0xfb10d4b8u, 0x9c47d08fu, 0xa6855419u, 0xfd17b448u,
                                0x0e1108a8u, 0x5da4fbfcu, 0x26a3c465u, 0x483ada77u};

static void pr_jac(const Jac26& P) {
    pr(P.X);
    pr(P.Y);
    pr(P.Z);
    printf(" %d\n", P.inf ? 1 : 0);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 200;
    for (int it = 0; it < n; ++it) {
        const int mode = it % 3;
        fe26 a, b, r;
        const int ma = 1 + static_cast<int>(rnd() % 16), mb = 1 + static_cast<int>(rnd() % 16);
        rand_fe(a, ma, mode);
        rand_fe(b, mb, mode == 2 ? 1 : mode);
        fe26_mul(r, a, b);
        field_case("mul", a, b, r);
        fe26_sqr(r, a);
        field_case("sqr", a, a, r);
        rand_fe(a, 16, 1);
        fe26_sqr(r, a);
        field_case("sqr", a, a, r);
        rand_fe(a, 1 + static_cast<int>(rnd() % 30), mode);
        rand_fe(b, 1 + static_cast<int>(rnd() % 30), mode);
        fe26_add(r, a, b);
        field_case("add", a, b, r);
        rand_fe(b, 1 + static_cast<int>(rnd() % 15), mode);
        fe26_sub<16>(r, a, b);
        field_case("sub", a, b, r);
        fe26_copy(r, a);
        fe26_normalize(r);
        field_case("norm", a, a, r);
        fe26_copy(r, a);
        fe26_normalize_weak(r);
        field_case("weak", a, a, r);
        // zero tests: 0, p, 2p, k p at high magnitude
        fe26_zero(b);
        fe26_sub<8>(r, b, b);  // 8p
        printf("Z %d 1\n", fe26_is_zero(r) ? 1 : 0);
        printf("Z %d %d\n", fe26_is_zero(a) ? 1 : 0, 2);  // 2: the checker decides from the next line
        field_case("zchk", a, a, a);
        for (int i = 0; i < 10; ++i) a.v[i] = f26::plimb(i);
        a.m = 1;
        printf("Z %d 1\n", fe26_is_zero(a) ? 1 : 0);  // p
        fe26_add(r, a, a);
        printf("Z %d 1\n", fe26_is_zero(r) ? 1 : 0);  // 2p
        fe26_one(b);
        fe26_add(r, r, b);
        printf("Z %d 0\n", fe26_is_zero(r) ? 1 : 0);  // 2p + 1
    }
    // square roots of random squares
    for (int it = 0; it < 8; ++it) {
        fe26 a, s, r;
        rand_fe(a, 1, 0);
        fe26_sqr(s, a);
        fe26_sqrt_cand(r, s);
        fe26_normalize(r);
        field_case("sqrt", s, s, r);
    }
    // k * G, left-to-right double-and-madd over random and extreme k
    Aff26 G;
    fe26_from_words(G.x, kGx);
    fe26_from_words(G.y, kGy);
    for (int it = 0; it < 24; ++it) {
        uint32_t k[8];
        for (int i = 0; i < 8; ++i) k[i] = rnd();
        if (it == 0) { memset(k, 0, sizeof k); k[0] = 1; }
        if (it == 1) { memset(k, 0, sizeof k); k[0] = 2; }
        if (it == 2) { memset(k, 0xff, sizeof k); }
        if (it == 3) { memset(k, 0, sizeof k); k[0] = 3; }
        Jac26 acc;
        CurveK1x::set_inf(acc);
        for (int bit = 255; bit >= 0; --bit) {
            CurveK1x::dbl(acc, acc);
            if ((k[bit >> 5] >> (bit & 31)) & 1u) {
                Jac26 s;
                CurveK1x::madd(s, acc, G);
                acc = s;
            }
        }
        printf("P %08x%08x%08x%08x%08x%08x%08x%08x", k[7], k[6], k[5], k[4], k[3], k[2], k[1], k[0]);
        pr_jac(acc);
    }
    // special cases of madd / add
    Jac26 P, Q, R, I;
    CurveK1x::from_aff(P, G);
    CurveK1x::dbl(P, P);
    CurveK1x::dbl(P, P);  // 4G, Z != 1
    CurveK1x::set_inf(I);
    // madd: 4G + G, and (G-affine) into a point equal to G: P == Q, and P == -Q
    Jac26 Gj;
    CurveK1x::from_aff(Gj, G);
    CurveK1x::dbl(Q, Gj);          // 2G
    Jac26 G2;
    CurveK1x::madd(G2, Q, G);      // 3G
    printf("A madd_3G");
    pr_jac(G2);
    {
        Jac26 Gs;                  // G with a non-trivial Z: 2G then subtract G via madd with -G
        Aff26 nG;
        fe26_copy(nG.x, G.x);
        fe26_neg<2>(nG.y, G.y);
        fe26_normalize(nG.y);
        CurveK1x::madd(Gs, Q, nG);  // 2G - G = G, Z != 1
        CurveK1x::madd(R, Gs, G);   // G + G: doubling branch
        printf("A madd_dbl");
        pr_jac(R);
        CurveK1x::madd(R, Gs, nG);  // G - G: infinity
        printf("A madd_inf");
        pr_jac(R);
        CurveK1x::madd(R, I, G);    // inf + G
        printf("A madd_from_inf");
        pr_jac(R);
        CurveK1x::add(R, P, Q);     // 4G + 2G
        printf("A add_6G");
        pr_jac(R);
        CurveK1x::add(R, Gs, Gj);   // G + G (different Z)
        printf("A add_dbl");
        pr_jac(R);
        Jac26 nGs;
        fe26_copy(nGs.X, Gs.X);
        fe26_neg<11>(nGs.Y, Gs.Y);
        fe26_copy(nGs.Z, Gs.Z);
        nGs.inf = false;
        CurveK1x::add(R, Gj, nGs);  // G - G
        printf("A add_inf");
        pr_jac(R);
        CurveK1x::add(R, I, P);     // inf + 4G
        printf("A add_inf_l");
        pr_jac(R);
        CurveK1x::add(R, P, I);     // 4G + inf
        printf("A add_inf_r");
        pr_jac(R);
    }
    return 0;
}
