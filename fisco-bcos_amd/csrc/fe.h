// fe.h -- 256-bit modular arithmetic for gfx950, 8 x 32-bit limbs per lane (little-endian limbs).
//
// Two reduction strategies, chosen per modulus:
//  * FieldK1  -- secp256k1 base field p = 2^256 - 2^32 - 977.  512-bit Comba product
//                (v_mad_u64_u32 + v_addc_co_u32 per partial product), then a pseudo-Mersenne fold
//                T = L + H*(2^32 + 977).  Values are kept "weakly reduced" in [0, 2^256);
//                normalize() gives the canonical residue.
//  * Mont<P>  -- Comba-interleaved ("FIPS") Montgomery multiplication, R = 2^256, for the SM2
//                base field (m' = 1, one zero limb skipped) and both group orders.  Values in
//                Montgomery form, fully reduced (< m).
// Each partial product is one v_mad_u64_u32 whose carry-out feeds one v_addc_co_u32 (inline asm,
// so the compiler cannot fall back to compare-and-select carry detection).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fe_asm.h"

namespace bcosgpu {

struct fe {
    uint32_t v[8];
};

// acc(64) + c2(32) += a * b   -- 96-bit column accumulator of the generic Montgomery product (group
// orders only; the base-field products are the scheduled blocks of fe_asm.h).  gfx940+ require two
// wait states between a VALU write of an SGPR and a VALU read of it, and hipcc pads neither inside
// an asm string nor across its boundary: s_nop 1 after the carry write (read by the v_addc and,
// after the statement, possibly by hipcc's code) and, in BG_MADC_K, before the SGPR operand read.
#define BG_MADC(acc, c2, a, b)                                                                 \
    do {                                                                                       \
        uint64_t cc_;                                                                          \
        asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\ts_nop 1" \
                     : "+v"(acc), "=&s"(cc_), "+v"(c2)                                         \
                     : "v"(a), "v"(b));                                                        \
    } while (0)
// same with a compile-time constant multiplier (lives in an SGPR)
#define BG_MADC_K(acc, c2, a, k)                                                               \
    do {                                                                                       \
        uint64_t cc_;                                                                          \
        asm volatile("s_nop 1\n\tv_mad_u64_u32 %0, %1, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\ts_nop 1" \
                     : "+v"(acc), "=&s"(cc_), "+v"(c2)                                         \
                     : "v"(a), "s"(k));                                                        \
    } while (0)

// 32 x 32 -> 64-bit product in one v_mad_u64_u32 (instead of a v_mul_lo_u32 / v_mul_hi_u32 pair)
// (the carry-out of these writes is a junk SGPR pair: padded so hipcc's next instructions may reuse
// it at once)
__device__ __forceinline__ uint64_t mul_wide(uint32_t a, uint32_t b) {
    uint64_t r, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0\n\ts_nop 1" : "=v"(r), "=s"(cc) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint64_t mul_wide_k(uint32_t a, uint32_t k) {
    uint64_t r, cc;
    asm("s_nop 1\n\tv_mad_u64_u32 %0, %1, %2, %3, 0\n\ts_nop 1" : "=v"(r), "=s"(cc) : "v"(a), "s"(k));
    return r;
}

__device__ __forceinline__ void fe_copy(fe& r, const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = a.v[i];
}
__device__ __forceinline__ void fe_set(fe& r, const uint32_t k[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = k[i];
}
__device__ __forceinline__ void fe_zero(fe& r) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = 0;
}
__device__ __forceinline__ uint32_t fe_is_zero_raw(const fe& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.v[i];
    return o == 0;
}
__device__ __forceinline__ uint32_t fe_eq_raw(const fe& a, const fe& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
    return o == 0;
}
// r = c ? a : r   (per lane, branch-free)
__device__ __forceinline__ void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : r.v[i];
}
// 32-bit add/sub with carry: lower to v_add_co_u32 / v_addc_co_u32 / v_sub(b)_co_u32 chains
__device__ __forceinline__ uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
    unsigned int co;
    const uint32_t r = __builtin_addc(a, b, cin, &co);
    cout = co;
    return r;
}
__device__ __forceinline__ uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
    unsigned int bo;
    const uint32_t r = __builtin_subc(a, b, bin, &bo);
    bout = bo;
    return r;
}
// r = lane-in-mask ? a : r, as explicit v_cndmask_b32 (the compiler cannot turn a chain of these
// into an indexed scratch array access, which it otherwise does for per-lane table selects)
// (one statement, opened by the two wait states hipcc owes the v_cmp that usually just wrote the mask)
__device__ __forceinline__ void fe_cmov_mask(fe& r, const fe& a, uint64_t mask) {
    asm volatile("s_nop 1\n\t"
                 "v_cndmask_b32_e64 %0, %0, %8, %16\n\tv_cndmask_b32_e64 %1, %1, %9, %16\n\t"
                 "v_cndmask_b32_e64 %2, %2, %10, %16\n\tv_cndmask_b32_e64 %3, %3, %11, %16\n\t"
                 "v_cndmask_b32_e64 %4, %4, %12, %16\n\tv_cndmask_b32_e64 %5, %5, %13, %16\n\t"
                 "v_cndmask_b32_e64 %6, %6, %14, %16\n\tv_cndmask_b32_e64 %7, %7, %15, %16"
                 : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
                   "+v"(r.v[6]), "+v"(r.v[7])
                 : "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]),
                   "v"(a.v[7]), "s"(mask));
}
// a < b as 256-bit integers
__device__ __forceinline__ bool fe_lt(const fe& a, const fe& b) {
    uint32_t bw = 0, t;
#pragma unroll
    for (int i = 0; i < 8; ++i) t = subc32(a.v[i], b.v[i], bw, bw);
    (void)t;
    return bw != 0;
}
__device__ __forceinline__ bool fe_lt_k(const fe& a, const uint32_t* k) {
    uint32_t bw = 0, t;
#pragma unroll
    for (int i = 0; i < 8; ++i) t = subc32(a.v[i], k[i], bw, bw);
    (void)t;
    return bw != 0;
}
// r = a + b (mod 2^256), returns carry
__device__ __forceinline__ uint32_t fe_add_raw(fe& r, const fe& a, const fe& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = addc32(a.v[i], b.v[i], c, c);
    return c;
}
// r = a - b (mod 2^256), returns borrow
__device__ __forceinline__ uint32_t fe_sub_raw(fe& r, const fe& a, const fe& b) {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = subc32(a.v[i], b.v[i], bw, bw);
    return bw;
}
__device__ __forceinline__ uint32_t fe_sub_k(fe& r, const fe& a, const uint32_t* k) {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = subc32(a.v[i], k[i], bw, bw);
    return bw;
}
__device__ __forceinline__ uint32_t fe_add_k(fe& r, const fe& a, const uint32_t* k) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = addc32(a.v[i], k[i], c, c);
    return c;
}

// 256 x 256 -> 512-bit product and 256-bit square: the scheduled Comba blocks of fe_asm.h
__device__ __forceinline__ void mul_512(uint32_t r[16], const fe& a, const fe& b) { mul_512_asm(r, a.v, b.v); }
__device__ __forceinline__ void sqr_512(uint32_t r[16], const fe& a) { sqr_512_asm(r, a.v); }

// ============================================================================ secp256k1 base field
struct FieldK1 {
    // p = 2^256 - c, c = 2^32 + 977
    static constexpr uint32_t P[8] = {0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu,
                                      0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};

    // r += f * c for f in {0, 1}; returns the carry out of 2^256
    __device__ static __forceinline__ uint32_t add_fc(fe& r, uint32_t f) {
        uint32_t c = 0;
        r.v[0] = addc32(r.v[0], f * 977u, 0, c);
        r.v[1] = addc32(r.v[1], f, c, c);
#pragma unroll
        for (int i = 2; i < 8; ++i) r.v[i] = addc32(r.v[i], 0u, c, c);
        return c;
    }
    // r -= f * c for f in {0, 1}; returns the borrow
    __device__ static __forceinline__ uint32_t sub_fc(fe& r, uint32_t f) {
        uint32_t b = 0;
        r.v[0] = subc32(r.v[0], f * 977u, 0, b);
        r.v[1] = subc32(r.v[1], f, b, b);
#pragma unroll
        for (int i = 2; i < 8; ++i) r.v[i] = subc32(r.v[i], 0u, b, b);
        return b;
    }

    // reduce a 512-bit value T = L + H 2^256 to [0, 2^256):  T = L + H*977 + H*2^32 (mod p)
    __device__ static __forceinline__ void reduce(fe& o, const uint32_t t[16]) { k1_reduce_asm(o.v, t); }

    __device__ static __forceinline__ void mul(fe& r, const fe& a, const fe& b) {
        uint32_t t[16];
        mul_512(t, a, b);
        reduce(r, t);
    }
    __device__ static __forceinline__ void sqr(fe& r, const fe& a) {
        uint32_t t[16];
        sqr_512(t, a);
        reduce(r, t);
    }
    __device__ static __forceinline__ void add(fe& r, const fe& a, const fe& b) { k1_add_asm(r.v, a.v, b.v); }
    __device__ static __forceinline__ void sub(fe& r, const fe& a, const fe& b) { k1_sub_asm(r.v, a.v, b.v); }
    // r = 2^K a, r = 3a: one shifted pass and one fold instead of K (or 2) full additions
    template <int K>
    __device__ static __forceinline__ void shl(fe& r, const fe& a) {
        static_assert(K >= 1 && K <= 3, "shift 1..3");
        if (K == 1) k1_shl1_asm(r.v, a.v);
        else if (K == 2) k1_shl2_asm(r.v, a.v);
        else k1_shl3_asm(r.v, a.v);
    }
    __device__ static __forceinline__ void mul3(fe& r, const fe& a) { k1_add_shl1_asm(r.v, a.v, a.v); }
    // canonical residue in [0, p)
    __device__ static __forceinline__ void normalize(fe& a) {
        fe t;
        k1_normalize_asm(t.v, a.v);
        fe_copy(a, t);
    }
    __device__ static __forceinline__ bool is_zero(const fe& a) {
        fe t;
        fe_copy(t, a);
        normalize(t);
        return fe_is_zero_raw(t);
    }
    __device__ static __forceinline__ bool eq(const fe& a, const fe& b) {
        fe t;
        sub(t, a, b);
        return is_zero(t);
    }
    __device__ static __forceinline__ void neg(fe& r, const fe& a) {
        fe z;
        fe_zero(z);
        sub(r, z, a);
    }
    __device__ static __forceinline__ void from_plain(fe& r, const fe& a) { fe_copy(r, a); }
    __device__ static __forceinline__ void to_plain(fe& r, const fe& a) {
        fe_copy(r, a);
        normalize(r);
    }
    __device__ static __forceinline__ void set_one(fe& r) {
        fe_zero(r);
        r.v[0] = 1;
    }
    __device__ static __forceinline__ void sqr_n(fe& r, const fe& a, int n) {
        sqr(r, a);
        for (int i = 1; i < n; ++i) sqr(r, r);
    }
    // x^(2^223 - 1) building blocks of libsecp256k1-style addition chains
    __device__ static __forceinline__ void chain223(fe& x223, fe& x22, fe& x2, fe& x3, const fe& a) {
        fe t, x6, x9, x11, x44, x88, x176, x220;
        sqr(t, a); mul(x2, t, a);
        sqr(t, x2); mul(x3, t, a);
        sqr_n(t, x3, 3); mul(x6, t, x3);
        sqr_n(t, x6, 3); mul(x9, t, x3);
        sqr_n(t, x9, 2); mul(x11, t, x2);
        sqr_n(t, x11, 11); mul(x22, t, x11);
        sqr_n(t, x22, 22); mul(x44, t, x22);
        sqr_n(t, x44, 44); mul(x88, t, x44);
        sqr_n(t, x88, 88); mul(x176, t, x88);
        sqr_n(t, x176, 44); mul(x220, t, x44);
        sqr_n(t, x220, 3); mul(x223, t, x3);
    }
    // a^(p-2)
    __device__ static __forceinline__ void inv(fe& r, const fe& a) {
        fe x223, x22, x2, x3, t;
        chain223(x223, x22, x2, x3, a);
        sqr_n(t, x223, 23); mul(t, t, x22);
        sqr_n(t, t, 5); mul(t, t, a);
        sqr_n(t, t, 3); mul(t, t, x2);
        sqr_n(t, t, 2); mul(r, t, a);
    }
    // a^((p+1)/4): a square root when one exists
    __device__ static __forceinline__ void sqrt_cand(fe& r, const fe& a) {
        fe x223, x22, x2, x3, t;
        chain223(x223, x22, x2, x3, a);
        sqr_n(t, x223, 23); mul(t, t, x22);
        sqr_n(t, t, 6); mul(t, t, x2);
        sqr_n(r, t, 2);
    }
};

// ============================================================================ Montgomery fields
struct ParamP2 {  // SM2 base field
    static constexpr bool SM2P = true;
    static constexpr uint32_t M[8] = {0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu,
                                      0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu};
    static constexpr uint32_t MINV = 0x1u;
    static constexpr uint32_t R2[8] = {0x00000003u, 0x00000002u, 0xffffffffu, 0x00000002u,
                                       0x00000001u, 0x00000001u, 0x00000002u, 0x00000004u};
    static constexpr uint32_t ONE[8] = {0x00000001u, 0x00000000u, 0xffffffffu, 0x00000000u,
                                        0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u};
    static constexpr uint32_t EXP_INV[8] = {0xfffffffdu, 0xffffffffu, 0x00000000u, 0xffffffffu,
                                            0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu};
};
struct ParamN1 {  // secp256k1 group order
    static constexpr bool SM2P = false;
    static constexpr uint32_t M[8] = {0xd0364141u, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u,
                                      0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    static constexpr uint32_t MINV = 0x5588b13fu;
    static constexpr uint32_t R2[8] = {0x67d7d140u, 0x896cf214u, 0x0e7cf878u, 0x741496c2u,
                                       0x5bcd07c6u, 0xe697f5e4u, 0x81c69bc5u, 0x9d671cd5u};
    static constexpr uint32_t ONE[8] = {0x2fc9bebfu, 0x402da173u, 0x50b75fc4u, 0x45512319u,
                                        0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u};
    static constexpr uint32_t EXP_INV[8] = {0xd036413fu, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u,
                                            0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
};
struct ParamN2 {  // SM2 group order
    static constexpr bool SM2P = false;
    static constexpr uint32_t M[8] = {0x39d54123u, 0x53bbf409u, 0x21c6052bu, 0x7203df6bu,
                                      0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu};
    static constexpr uint32_t MINV = 0x72350975u;
    static constexpr uint32_t R2[8] = {0x7c114f20u, 0x901192afu, 0xde6fa2fau, 0x3464504au,
                                       0x3affe0d4u, 0x620fc84cu, 0xa22b3d3bu, 0x1eb5e412u};
    static constexpr uint32_t ONE[8] = {0xc62abeddu, 0xac440bf6u, 0xde39fad4u, 0x8dfc2094u,
                                        0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u};
    static constexpr uint32_t EXP_INV[8] = {0x39d54121u, 0x53bbf409u, 0x21c6052bu, 0x7203df6bu,
                                            0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu};
};

// Montgomery reduction specialised to the SM2 prime p = 2^256 - 2^224 - 2^96 + 2^64 - 1 (m' = 1):
// adding q p 2^(32i) to the 512-bit T puts +q at word i+8, -q at i+7, -q at i+3, +q at i+2 and
// clears word i (q = its current value), so the reduction needs no multiplications: a column sweep
// with a signed 64-bit accumulator (v_lshl_add_u64 adds).  T < p^2 -> result < 2p -> one conditional
// subtraction.  Replaces the 56 multiply-accumulates of the generic CIOS reduction.
__device__ __forceinline__ void redc_sm2p(fe& r, const uint32_t t[16]) {
    uint32_t q[8], o[8];
    int64_t acc = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        acc += static_cast<int64_t>(t[c]);
        if (c >= 2 && c <= 9) acc += static_cast<int64_t>(q[c - 2]);
        if (c >= 8) acc += static_cast<int64_t>(q[c - 8]);
        int64_t neg = 0;
        if (c >= 3 && c <= 10) neg += static_cast<int64_t>(q[c - 3]);
        if (c >= 7 && c <= 14) neg += static_cast<int64_t>(q[c - 7]);
        acc -= neg;
        if (c < 8) {
            q[c] = static_cast<uint32_t>(acc);
            acc -= static_cast<int64_t>(q[c]);
        } else {
            o[c - 8] = static_cast<uint32_t>(acc);
        }
        acc >>= 32;
    }
    const uint32_t top = static_cast<uint32_t>(acc);  // 0 or 1
    fe t2, u;
#pragma unroll
    for (int i = 0; i < 8; ++i) t2.v[i] = o[i];
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) u.v[i] = subc32(t2.v[i], ParamP2::M[i], bw, bw);
    const bool take = top != 0u || bw == 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = take ? u.v[i] : t2.v[i];
}

template <class P>
struct Mont {
    static constexpr const uint32_t* M = P::M;

    // r = a * b * 2^-256 mod m (inputs < m, output < m)
    __device__ static __forceinline__ void mul(fe& r, const fe& a, const fe& b) {
        if constexpr (P::SM2P) {
            uint32_t t[16];
            mul_512(t, a, b);
            redc_sm2p(r, t);
            return;
        }
        uint64_t acc = 0;
        uint32_t c2 = 0, m[8], o[8];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int j = k - i;
                if (j >= 0 && j < 8) BG_MADC(acc, c2, a.v[i], b.v[j]);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int j = k - i;
                if (i < k && j >= 1 && j < 8 && P::M[j] != 0u) BG_MADC_K(acc, c2, m[i], P::M[j]);
            }
            if (k < 8) {
                m[k] = P::MINV == 1u ? static_cast<uint32_t>(acc) : static_cast<uint32_t>(acc) * P::MINV;
                BG_MADC_K(acc, c2, m[k], P::M[0]);
            } else {
                o[k - 8] = static_cast<uint32_t>(acc);
            }
            acc = (acc >> 32) | (static_cast<uint64_t>(c2) << 32);
            c2 = 0;
        }
        // result = o + top * 2^256 < 2m ; subtract m once if needed
        const uint32_t top = static_cast<uint32_t>(acc);
        fe t, u;
#pragma unroll
        for (int i = 0; i < 8; ++i) t.v[i] = o[i];
        const uint32_t bw = fe_sub_k(u, t, P::M);
        const bool take = top != 0u || bw == 0u;
#pragma unroll
        for (int i = 0; i < 8; ++i) r.v[i] = take ? u.v[i] : t.v[i];
    }
    __device__ static __forceinline__ void sqr(fe& r, const fe& a) {
        if constexpr (P::SM2P) {
            uint32_t t[16];
            sqr_512(t, a);
            redc_sm2p(r, t);
        } else {
            mul(r, a, a);
        }
    }
    __device__ static __forceinline__ void add(fe& r, const fe& a, const fe& b) { mod_add_asm(r.v, a.v, b.v, P::M); }
    __device__ static __forceinline__ void sub(fe& r, const fe& a, const fe& b) { mod_sub_asm(r.v, a.v, b.v, P::M); }
    template <int K>
    __device__ static __forceinline__ void shl(fe& r, const fe& a) {
        add(r, a, a);
#pragma unroll
        for (int k = 1; k < K; ++k) add(r, r, r);
    }
    __device__ static __forceinline__ void mul3(fe& r, const fe& a) {
        fe t;
        add(t, a, a);
        add(r, t, a);
    }
    __device__ static __forceinline__ void neg(fe& r, const fe& a) {
        fe z;
        fe_zero(z);
        sub(r, z, a);
    }
    __device__ static __forceinline__ void normalize(fe&) {}
    __device__ static __forceinline__ bool is_zero(const fe& a) { return fe_is_zero_raw(a); }
    __device__ static __forceinline__ bool eq(const fe& a, const fe& b) { return fe_eq_raw(a, b); }
    __device__ static __forceinline__ void set_one(fe& r) { fe_set(r, P::ONE); }
    // plain (< m) -> Montgomery form
    __device__ static __forceinline__ void from_plain(fe& r, const fe& a) {
        fe k;
        fe_set(k, P::R2);
        mul(r, a, k);
    }
    __device__ static __forceinline__ void to_plain(fe& r, const fe& a) {
        fe one;
        fe_zero(one);
        one.v[0] = 1;
        mul(r, a, one);
    }
    __device__ static __forceinline__ void sqr_n(fe& r, const fe& a, int n) {
        sqr(r, a);
        for (int i = 1; i < n; ++i) sqr(r, r);
    }
    // a^(m-2) for the group orders: their top 128 bits are [127 ones][0] (secp256k1 n) or
    // [31 ones][0][96 ones] (SM2 n), done by x^(2^k - 1) chains; the low 128 bits by a
    // square-and-multiply loop whose branch is wave-uniform (the exponent is a constant).
    __device__ static __forceinline__ void inv(fe& r, const fe& a) {
        fe x2, x3, x6, x12, x24, x31, x32, x48, x96, t;
        sqr(t, a); mul(x2, t, a);
        sqr(t, x2); mul(x3, t, a);
        sqr_n(t, x3, 3); mul(x6, t, x3);
        sqr_n(t, x6, 6); mul(x12, t, x6);
        sqr_n(t, x12, 12); mul(x24, t, x12);
        sqr_n(t, x24, 6); mul(t, t, x6);
        sqr(t, t); mul(x31, t, a);
        sqr(t, x31); mul(x32, t, a);
        sqr_n(t, x24, 24); mul(x48, t, x24);
        sqr_n(t, x48, 48); mul(x96, t, x48);
        if (P::EXP_INV[7] == 0xffffffffu) {  // secp256k1 n: [127 ones][0]
            fe x120, x126;
            sqr_n(t, x96, 24); mul(x120, t, x24);
            sqr_n(t, x120, 6); mul(x126, t, x6);
            sqr(t, x126); mul(t, t, a);  // 127 ones
            sqr(r, t);                   // 0
        } else {  // SM2 n: [31 ones][0][96 ones]
            sqr(t, x31);
            sqr_n(t, t, 96); mul(r, t, x96);
        }
#pragma unroll 1
        for (int bit = 127; bit >= 0; --bit) {
            sqr(r, r);
            if ((P::EXP_INV[bit >> 5] >> (bit & 31)) & 1u) mul(r, r, a);
        }
    }
};

using FieldN1 = Mont<ParamN1>;
using FieldN2 = Mont<ParamN2>;

// SM2 base field: Montgomery arithmetic plus an addition chain for p - 2 =
// [31 ones][0][128 ones][32 zeros][32 ones][30 ones][0][1]  (255 S + 13 M)
struct FieldP2 : Mont<ParamP2> {
    __device__ static __forceinline__ void inv(fe& r, const fe& a) {
        fe x2, x3, x6, x12, x15, x30, x31, x32, x64, x128, t;
        sqr(t, a); mul(x2, t, a);
        sqr(t, x2); mul(x3, t, a);
        sqr_n(t, x3, 3); mul(x6, t, x3);
        sqr_n(t, x6, 6); mul(x12, t, x6);
        sqr_n(t, x12, 3); mul(x15, t, x3);
        sqr_n(t, x15, 15); mul(x30, t, x15);
        sqr(t, x30); mul(x31, t, a);
        sqr(t, x31); mul(x32, t, a);
        sqr_n(t, x32, 32); mul(x64, t, x32);
        sqr_n(t, x64, 64); mul(x128, t, x64);
        sqr(t, x31);                        // [31 ones][0]
        sqr_n(t, t, 128); mul(t, t, x128);  // [128 ones]
        sqr_n(t, t, 32);                    // [32 zeros]
        sqr_n(t, t, 32); mul(t, t, x32);    // [32 ones]
        sqr_n(t, t, 30); mul(t, t, x30);    // [30 ones]
        sqr_n(t, t, 2); mul(r, t, a);       // [0][1]
    }
};

// ---------------------------------------------------------------- byte conversions
// 32 big-endian bytes (8 little-endian-loaded words w[0..7] in memory order) -> limbs
__device__ __forceinline__ void fe_from_be_words(fe& r, const uint32_t w[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = __builtin_bswap32(w[7 - i]);
}
__device__ __forceinline__ void fe_to_be_words(uint32_t w[8], const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[7 - i] = __builtin_bswap32(a.v[i]);
}

}  // namespace bcosgpu
