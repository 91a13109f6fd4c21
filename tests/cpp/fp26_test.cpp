// fp26_test.cpp -- host build of fp26.h / ecp26.h (SM2, Montgomery R = 2^286) with FE26_CHECK: every
// magnitude contract and limb bound asserted at run time; tests/test_fp26.py recomputes the results with
// Python integers.  Lines:
//   F <op> <a limbs> <b limbs> <r limbs>      field cases (mul/sqr: Montgomery products)
//   Z <got> <want>                            zero tests (want 2: decided from the next F zchk line)
//   P <k hex> <X> <Y> <Z> <inf>               k*G (Montgomery coordinates) by double-and-madd
//   A <case> <X> <Y> <Z> <inf>                madd / add special cases
#define FE26_CHECK 1
#include "../../fisco-bcos_amd/csrc/ecp26.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

using namespace bcosgpu;

static uint64_t rng = 0x2545f4914f6cdd1dull;
static uint32_t rnd() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return static_cast<uint32_t>(rng >> 11);
}
static void rand_fp(fp26& a, int m, int mode) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t bound = static_cast<uint64_t>(m) << (i == 9 ? 22 : 26);
        uint64_t v;
        if (mode == 1) v = bound;
        else if (mode == 2) v = (i == static_cast<int>(rnd() % 10)) ? bound : 0;
        else v = ((static_cast<uint64_t>(rnd()) << 20) ^ rnd()) % (bound + 1);
        a.v[i] = static_cast<uint32_t>(v);
    }
    a.m = m;
}
static void pr(const fp26& a) {
    for (int i = 0; i < 10; ++i) printf("%s%x", i ? "," : " ", a.v[i]);
}
static void fcase(const char* op, const fp26& a, const fp26& b, const fp26& r) {
    printf("F %s", op);
    pr(a);
    pr(b);
    pr(r);
    printf("\n");
}
static void pr_jac(const JacP26& P) {
    pr(P.X);
    pr(P.Y);
    pr(P.Z);
    printf(" %d\n", P.inf ? 1 : 0);
}
// G plain words (little-endian)
static const uint32_t kGx[8] = {0x334c74c7u, 0x715a4589u, 0xf2660be1u, 0x8fe30bbfu,
                                0x6a39c994u, 0x5f990446u, 0x1f198119u, 0x32c4ae2cu};
static const uint32_t kGy[8] = {0x2139f0a0u, 0x02df32e5u, 0xc62a4740u, 0xd0a9877cu,
                                0x6b692153u, 0x59bdcee3u, 0xf4f6779cu, 0xbc3736a2u};

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 150;
    for (int it = 0; it < n; ++it) {
        const int mode = it % 3;
        fp26 a, b, r;
        rand_fp(a, 1 + static_cast<int>(rnd() % 15), mode);
        rand_fp(b, 1 + static_cast<int>(rnd() % 15), mode == 2 ? 1 : mode);
        fp26_mul(r, a, b);
        fcase("mul", a, b, r);
        fp26_sqr(r, a);
        fcase("sqr", a, a, r);
        rand_fp(a, 15, 1);  // every limb at the contract's bound
        fp26_sqr(r, a);
        fcase("sqr", a, a, r);
        rand_fp(b, 15, 1);
        fp26_mul(r, a, b);
        fcase("mul", a, b, r);
        rand_fp(a, 1 + static_cast<int>(rnd() % 30), mode);
        rand_fp(b, 1 + static_cast<int>(rnd() % 30), mode);
        fp26_add(r, a, b);
        fcase("add", a, b, r);
        rand_fp(a, 1 + static_cast<int>(rnd() % 20), mode);
        rand_fp(b, 1 + static_cast<int>(rnd() % 15), mode);
        fp26_sub<16>(r, a, b);
        fcase("sub", a, b, r);
        fp26_neg<16>(r, b);
        fcase("neg", b, b, r);
        fp26_copy(r, a);
        fp26_normalize(r);
        fcase("norm", a, a, r);
        fp26_copy(r, a);
        fp26_normalize_weak(r);
        fcase("weak", a, a, r);
        printf("Z %d 2\n", fp26_is_zero(a) ? 1 : 0);
        fcase("zchk", a, a, a);
        fp26 z;
        fp26_zero(z);
        fp26_sub<8>(r, z, z);  // 8p
        printf("Z %d 1\n", fp26_is_zero(r) ? 1 : 0);
        fp26_set(a, p26::P);
        printf("Z %d 1\n", fp26_is_zero(a) ? 1 : 0);  // p
        fp26_add(r, a, a);
        printf("Z %d 1\n", fp26_is_zero(r) ? 1 : 0);  // 2p
        fp26_set(b, p26::ONE_R);
        fp26_add(r, r, b);
        printf("Z %d 0\n", fp26_is_zero(r) ? 1 : 0);  // 2p + R
    }
    // k*G, left-to-right double-and-madd, in the Montgomery domain
    AffP26 G;
    fp26 gx, gy;
    fp26_from_words(gx, kGx);
    fp26_from_words(gy, kGy);
    fp26_to_mont(G.x, gx);
    fp26_to_mont(G.y, gy);
    for (int it = 0; it < 20; ++it) {
        uint32_t k[8];
        for (int i = 0; i < 8; ++i) k[i] = rnd();
        if (it == 0) { memset(k, 0, sizeof k); k[0] = 1; }
        if (it == 1) { memset(k, 0, sizeof k); k[0] = 2; }
        if (it == 2) { memset(k, 0xff, sizeof k); }
        JacP26 acc;
        CurveSM2x::set_inf(acc);
        for (int bit = 255; bit >= 0; --bit) {
            CurveSM2x::dbl(acc, acc);
            if ((k[bit >> 5] >> (bit & 31)) & 1u) {
                JacP26 s;
                CurveSM2x::madd(s, acc, G);
                acc = s;
            }
        }
        printf("P %08x%08x%08x%08x%08x%08x%08x%08x", k[7], k[6], k[5], k[4], k[3], k[2], k[1], k[0]);
        pr_jac(acc);
    }
    // special cases
    JacP26 P4, Q2, R, I, Gj, Gs;
    CurveSM2x::from_aff(Gj, G);
    CurveSM2x::dbl(Q2, Gj);   // 2G
    CurveSM2x::dbl(P4, Q2);   // 4G
    CurveSM2x::set_inf(I);
    AffP26 nG;
    fp26_copy(nG.x, G.x);
    fp26_neg<2>(nG.y, G.y);
    fp26_normalize(nG.y);
    CurveSM2x::madd(Gs, Q2, nG);  // G with Z != 1
    printf("A madd_G");
    pr_jac(Gs);
    CurveSM2x::madd(R, Gs, G);   // doubling branch
    printf("A madd_dbl");
    pr_jac(R);
    CurveSM2x::madd(R, Gs, nG);  // infinity
    printf("A madd_inf");
    pr_jac(R);
    CurveSM2x::madd(R, I, G);
    printf("A madd_from_inf");
    pr_jac(R);
    CurveSM2x::add(R, P4, Q2);   // 6G
    printf("A add_6G");
    pr_jac(R);
    CurveSM2x::add(R, Gs, Gj);   // 2G via the doubling branch
    printf("A add_dbl");
    pr_jac(R);
    JacP26 nGs = Gs;
    fp26_neg<12>(nGs.Y, Gs.Y);  // Gs.Y <= 11 (madd)
    fp26_normalize_weak(nGs.Y);
    CurveSM2x::add(R, Gj, nGs);  // infinity
    printf("A add_inf");
    pr_jac(R);
    CurveSM2x::add(R, I, P4);
    printf("A add_inf_l");
    pr_jac(R);
    CurveSM2x::add(R, P4, I);
    printf("A add_inf_r");
    pr_jac(R);
    return 0;
}
