// fp26.h -- the SM2 base field p = 2^256 - 2^224 - 2^96 + 2^64 - 1 in ten 26-bit limbs with lazy carries,
// Montgomery form with R = 2^286 (an element x is stored as x R mod p).  The SM2 counterpart of fe26.h,
// for the same reason: a lone wave (the small-batch pair kernel) spends most of its time in VCC carry
// chains with the 8 x 32-bit representation; here additions are independent limb adds.
//
// Reduction.  -p^-1 = 1 (mod 2^26) (p = -1 mod 2^64), so the Montgomery digit of column i is simply its
// low 26 bits m, and adding m p 2^(26i) through p's sparse form clears column i and adds
//   +m 2^12 to column i+2 (2^64 = 2^(2*26+12)),   -m 2^18 to column i+3 (2^96),
//   -m 2^16 to column i+8 (2^224),                 +m 2^22 to column i+9 (2^256):
// four multiply-adds by constants per digit, no multiply by p's limbs.  Columns are signed 64-bit
// accumulators.  Eleven digits (R = 2^286 rather than 2^260) make the output (T + M p) / R < T / R + p
// < p + 2^234 for inputs of magnitude <= 15, i.e. magnitude 1 whatever the inputs (limb 9 <= 2^22).
// Why 15: the largest column is column 8, nine products of limbs <= m 2^26 (limb 9, <= m 2^22, is not in
// it; column 9's two limb-9 products are 2^4 smaller): 9 m^2 2^52 = 2025 * 2^52 < 2^63 - 2^56.5 at
// m = 15, and the redc terms (carry < 2^37, digit terms < 2^49) stay inside that headroom; at m = 16 the
// column could reach 2^63.2 and wrap.
//
// Magnitude (as fe26.h: limbs 0..8 <= m 2^26, limb 9 <= m 2^22):
//   mul, sqr       : inputs m <= 15 (every column stays < 2^63 signed, see above) -> m = 1
//   add            : m_a + m_b                 (<= 63)
//   sub<K>         : m_b <= K - 1              -> m_a + K + 1  (K p in limbs each >= (K-1) 2^26)
//   neg<K>         : m <= K - 1                -> K + 1
//   mul_int<C>     : m * C
//   normalize_weak : any m <= 63               -> 2
//   normalize      : any m <= 63               -> canonical
// The host build with FE26_CHECK (tests/cpp/fp26_test.cpp) asserts them.
#pragma once
#include "fe26.h"

namespace bcosgpu {

struct fp26 {
    uint32_t v[10];
    F26_FIELD_M
};

namespace p26 {
constexpr uint32_t M26 = 0x3ffffffu, M22 = 0x3fffffu;
constexpr uint32_t P[10] = {0x3ffffffu, 0x3ffffffu, 0xfffu,     0x3fc0000u, 0x3ffffffu,
                            0x3ffffffu, 0x3ffffffu, 0x3ffffffu, 0x3feffffu, 0x3fffffu};
// limb i of K p written with every limb i <= 8 in [K 2^26 - K, (K + 1) 2^26): standard limbs s_i of K p,
// plus K 2^26 borrowed from the next limb
F26_HD constexpr uint32_t kp_std(int K, int i) {
    uint64_t c = 0, s = 0;
    for (int j = 0; j <= i; ++j) {
        const uint64_t t = static_cast<uint64_t>(K) * P[j] + c;
        s = j < 9 ? (t & M26) : t;
        c = t >> 26;
    }
    return static_cast<uint32_t>(s);
}
F26_HD constexpr uint32_t kp(int K, int i) {
    return i == 0 ? kp_std(K, 0) + static_cast<uint32_t>(K) * (1u << 26)
         : i < 9  ? kp_std(K, i) + static_cast<uint32_t>(K) * (1u << 26) - static_cast<uint32_t>(K)
                  : kp_std(K, 9) - static_cast<uint32_t>(K);
}
// R mod p and R^2 mod p (R = 2^286), limbs
constexpr uint32_t ONE_R[10] = {0x0u, 0x10u, 0x0u, 0x3ff0000u, 0x3fffffu, 0x0u, 0x0u, 0x0u, 0x0u, 0x100000u};
constexpr uint32_t R2[10] = {0x0u, 0x10u, 0x300u, 0x3ff8000u, 0x2fffffu, 0x0u, 0x3u, 0x40u, 0x1000u, 0x180000u};
// R^3 mod p: (x R)^-1 (a plain inverse) times R^3 in the Montgomery product gives x^-1 R
constexpr uint32_t R3[10] = {0x0u, 0x24u, 0x6c0u, 0x3ff2000u, 0x6bffffu, 0x3000000u, 0x4u, 0xf0u, 0x3000u, 0x2e0000u};
// b R mod p
constexpr uint32_t B_R[10] = {0x103f862u, 0xdd422u, 0x13b6cafu, 0x1336cc2u, 0x2c37146u,
                              0x31cf379u, 0x29470f1u, 0x181505eu, 0x114149eu, 0xde30cu};
}  // namespace p26

#ifdef FE26_CHECK
F26_HD void fp26_check(const fp26& a) {
    assert(a.m >= 1 && a.m <= 63);
    for (int i = 0; i < 9; ++i) assert((uint64_t)a.v[i] <= (uint64_t)a.m << 26);
    assert((uint64_t)a.v[9] <= (uint64_t)a.m << 22);
}
#define P26_CHK(a) fp26_check(a)
#else
#define P26_CHK(a) ((void)0)
#endif

F26_HD void fp26_copy(fp26& r, const fp26& a) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = a.v[i];
    F26_SETM(r, a.m);
}
F26_HD void fp26_set(fp26& r, const uint32_t k[10]) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = k[i];
    F26_SETM(r, 1);
}
F26_HD void fp26_zero(fp26& r) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = 0;
    F26_SETM(r, 1);
}
// plain words (< 2^256) -> limbs of the same integer (not yet in Montgomery form)
F26_HD void fp26_from_words(fp26& r, const uint32_t w[8]) {
    fe26 t;
    fe26_from_words(t, w);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = t.v[i];
    F26_SETM(r, 1);
}
F26_HD void fp26_to_words(uint32_t w[8], const fp26& a) {  // a canonical
    fe26 t;
#pragma unroll
    for (int i = 0; i < 10; ++i) t.v[i] = a.v[i];
    fe26_to_words(w, t);
}

// Montgomery reduction of the 19 product columns (see the header): r = T 2^-286 mod p, m = 1
F26_HD void fp26_redc(fp26& r, int64_t c[21]) {
    using namespace p26;
    c[19] = 0;
    c[20] = 0;
#pragma unroll
    for (int i = 0; i < 11; ++i) {
        const int64_t t = c[i];
        const int64_t m = static_cast<int64_t>(static_cast<uint32_t>(t) & M26);
        c[i + 1] += t >> 26;  // floor((t - m) / 2^26): column i is now exactly zero
        c[i + 2] += m << 12;
        c[i + 3] -= m << 18;
        c[i + 8] -= m << 16;
        c[i + 9] += m << 22;
    }
#pragma unroll
    for (int j = 11; j < 20; ++j) {
        const int64_t t = c[j];
        r.v[j - 11] = static_cast<uint32_t>(t) & M26;
        c[j + 1] += t >> 26;
    }
    r.v[9] = static_cast<uint32_t>(c[20]);
    F26_SETM(r, 1);
}

F26_HD void fp26_mul(fp26& r, const fp26& a, const fp26& b) {
    F26_REQ(a.m <= 15 && b.m <= 15);
    P26_CHK(a);
    P26_CHK(b);
#if F26_ASM
    fp26_mul_asm(r.v, a.v, b.v);  // fe_asm.h: the same columns and digits, generated and scheduled
    return;
#endif
    int64_t c[21];
#pragma unroll
    for (int k = 0; k < 19; ++k) {
        uint64_t s = 0;
#pragma unroll
        for (int i = (k < 10 ? 0 : k - 9); i <= (k < 10 ? k : 9); ++i)
            s += static_cast<uint64_t>(a.v[i]) * b.v[k - i];
        c[k] = static_cast<int64_t>(s);
    }
    fp26_redc(r, c);
    P26_CHK(r);
}

F26_HD void fp26_sqr(fp26& r, const fp26& a) {
    F26_REQ(a.m <= 15);
    P26_CHK(a);
#if F26_ASM
    fp26_sqr_asm(r.v, a.v);
    return;
#endif
    uint32_t d[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) d[i] = a.v[i] << 1;
    int64_t c[21];
#pragma unroll
    for (int k = 0; k < 19; ++k) {
        uint64_t s = 0;
        const int lo = k < 10 ? 0 : k - 9;
        const int hi = k < 10 ? k : 9;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            const int j = k - i;
            if (i < j) s += static_cast<uint64_t>(d[i]) * a.v[j];
            else if (i == j) s += static_cast<uint64_t>(a.v[i]) * a.v[i];
        }
        c[k] = static_cast<int64_t>(s);
    }
    fp26_redc(r, c);
    P26_CHK(r);
}

F26_HD void fp26_add(fp26& r, const fp26& a, const fp26& b) {
    F26_REQ(a.m + b.m <= 63);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
    F26_SETM(r, a.m + b.m);
    P26_CHK(r);
}

template <int K>
F26_HD void fp26_sub(fp26& r, const fp26& a, const fp26& b) {
    F26_REQ(b.m <= K - 1 && a.m + K + 1 <= 63);
    P26_CHK(a);
    P26_CHK(b);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + (p26::kp(K, i) - b.v[i]);
    F26_SETM(r, a.m + K + 1);
    P26_CHK(r);
}

template <int K>
F26_HD void fp26_neg(fp26& r, const fp26& a) {
    F26_REQ(a.m <= K - 1);
    P26_CHK(a);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = p26::kp(K, i) - a.v[i];
    F26_SETM(r, K + 1);
    P26_CHK(r);
}

template <int C>
F26_HD void fp26_mul_int(fp26& r, const fp26& a) {
    F26_REQ(a.m * C <= 63);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] * C;
    F26_SETM(r, a.m * C);
    P26_CHK(r);
}

// one carry pass and one fold of the bits at 2^256 and above (2^256 = 2^224 + 2^96 - 2^64 + 1):
// limbs 0..8 < 2^26, limb 9 < 2^22 + 2^5 (m = 2), value < 2^256 + 2^240; signed intermediates
F26_HD void fp26_normalize_weak(fp26& r) {
    using namespace p26;
    P26_CHK(r);
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = r.v[i];
    const int64_t x = t[9] >> 22;  // < 2^6 for m <= 63
    t[9] &= M22;
    t[0] += x;
    t[2] -= x << 12;
    t[3] += x << 18;
    t[8] += x << 16;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        t[i + 1] += t[i] >> 26;  // floor division: limb i into [0, 2^26)
        t[i] &= M26;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = static_cast<uint32_t>(t[i]);
    F26_SETM(r, 2);
    P26_CHK(r);
}

// canonical residue in [0, p)
F26_HD void fp26_normalize(fp26& r) {
    using namespace p26;
    fp26_normalize_weak(r);
    // value < 2^256 + 2^240: fold once more, then at most one subtraction of p
    int64_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = r.v[i];
    const int64_t x = t[9] >> 22;
    t[9] &= M22;
    t[0] += x;
    t[2] -= x << 12;
    t[3] += x << 18;
    t[8] += x << 16;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        t[i + 1] += t[i] >> 26;
        t[i] &= M26;
    }
    // now 0 <= value < 2^256; subtract p when value >= p: compute value - p with borrows
    int64_t u[10];
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int64_t d = t[i] - static_cast<int64_t>(P[i]) + br;
        u[i] = d & (i == 9 ? M22 : M26);
        br = d >> (i == 9 ? 22 : 26);
    }
    const bool ge = br >= 0;  // no borrow out of the top: value >= p
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = static_cast<uint32_t>(ge ? u[i] : t[i]);
    F26_SETM(r, 1);
}

// a == 0 (mod p): after the weak pass the value is < 2^256 + 2^240 < 2p, so it is 0 or p
F26_HD bool fp26_is_zero(const fp26& a) {
    fp26 t;
    fp26_copy(t, a);
    fp26_normalize_weak(t);
    uint32_t z0 = 0, z1 = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        z0 |= t.v[i];
        z1 |= t.v[i] ^ p26::P[i];
    }
    return z0 == 0u || z1 == 0u;
}

F26_HD void fp26_cmov(fp26& r, const fp26& a, bool c) {
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = c ? a.v[i] : r.v[i];
#ifdef FE26_CHECK
    r.m = a.m > r.m ? a.m : r.m;
#endif
}

// into / out of the Montgomery domain
F26_HD void fp26_to_mont(fp26& r, const fp26& a) {
    fp26 k;
    fp26_set(k, p26::R2);
    fp26_mul(r, a, k);
}
F26_HD void fp26_from_mont(fp26& r, const fp26& a) {  // canonical plain value
    fp26 one;
    fp26_zero(one);
    one.v[0] = 1;
    fp26_mul(r, a, one);
    fp26_normalize(r);
}

}  // namespace bcosgpu
