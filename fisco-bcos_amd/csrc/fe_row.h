// fe_row.h -- a secp256k1 base-field element spread over one 16-lane DPP row: lane k (k < 10) of the
// row holds limb k of the ten-limb, radix-2^26 form of fe26.h; lanes 10..15 hold 0.  For the latency
// kernels (one signature per wave, few waves per SIMD), where the chain of dependent products is the
// whole cost: a lone wave issues one wave64 instruction per ~4.3 cycles whatever its lanes do, so the
// one-lane fe26 product (174 instructions, 928 cycles per dependent product in tools/splitbench.hip)
// costs its instruction count.  Spread over a row, each lane computes ONE product column:
//   conv   ten steps of  acc += a_i * t,  a_i broadcast over the row (DPP row_newbcast:i) and t = b
//          rotated by one lane per step (row_ror:1), so lane k holds b_(k-i) at step i; columns 16..18
//          wrap into lanes 0..2 (their sources, lanes 10..15, hold 0 everywhere else) and are kept in a
//          second accumulator for the three steps where they occur;
//   reduce the 64-bit columns are carried in parallel (each lane splits its column into 26-bit pieces
//          sent one and two lanes up), the columns 10..20 fold with 2^260 = 2^36 + R0 (mod p) as
//          R0 * H_j into lane j and 2^10 * H_j into lane j + 1 (a lane shift by 10 / 6 lanes), one
//          more carry round, and the column-10/11 overflow folds once more into lanes 0..2;
// about 80 wave instructions and 10 multiplies per product, with four independent products per wave
// (one per row).  Additions, subtractions and small multiples are ONE lane-wise instruction.
//
// Magnitude m: every limb, limb 9 included, is <= m * B with B = 2^26 + 2^16 (value < m * 2^260.1):
//   mul, sqr : inputs m <= 16 (limbs < 2^30.01: a column < 10 * 2^60.02 < 2^63.4)  -> m = 1 (limbs 0..8
//              < 2^26 + 2^14, limb 9 < 2^26 + 2^15.1)
//   add      : m_a + m_b;  mul_int<C>: C m
//   sub<K>   : a + K Q - b with Q = 16 p in radix-2^26 digits (each within 2^-12 of 2^26, so K Q >= b
//              limb by limb when b.m <= K - 1)  -> m_a + K
// the same contracts as fe26.h's, so ec_row.h's point formulas keep ec26.h's magnitude schedule.
// The bounds are checked by tools/rowbench.hip on the GPU (every product of every chain, lanes 10..15
// zero, limbs under the stated bound) and the results against fe26's one-lane products.
#pragma once
#include <stdint.h>

namespace bcosgpu {
namespace frow {

constexpr uint32_t M26 = 0x3ffffffu;
constexpr uint32_t R0 = 0x3d10u;  // 2^260 = 2^36 + R0 (mod p)

// DPP moves within a 16-lane row; a source lane outside the row reads 0 (bound_ctrl)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, true));
}
template <int N>
__device__ __forceinline__ uint32_t shl(uint32_t v) { return dpp<0x100 + N>(v); }  // lane i <- lane i + N
template <int N>
__device__ __forceinline__ uint32_t shr(uint32_t v) { return dpp<0x110 + N>(v); }  // lane i <- lane i - N
template <int N>
__device__ __forceinline__ uint32_t ror(uint32_t v) { return dpp<0x120 + N>(v); }  // lane i <- lane (i - N) mod 16
template <int N>
__device__ __forceinline__ uint32_t bcast(uint32_t v) { return dpp<0x150 + N>(v); }  // every lane <- lane N

// A value the compiler cannot see through: lane masks built from it stay bitwise operations (a select
// on a lane-dependent condition may otherwise become an EXEC branch, and a DPP move under a partial EXEC
// would read the disabled lanes as 0).
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t mask_if(bool c) { return opaque(c ? 0xffffffffu : 0u); }

// the row's constants: lane k, the row in the wave, Q's digit for this lane (0 on lanes 10..15), and the
// lane masks of the product and of the per-row operand choice
struct Lane {
    int k, row;
    uint32_t q, one;
    uint32_t ge3, eq15, ge14, lt10, lt9, keep9;  // keep9: M26 on lanes 0..8, all ones elsewhere
    uint32_t r0, r1, r2;                    // row == 0, 1, 2
    __device__ __forceinline__ explicit Lane(int lane) : k(lane & 15), row((lane >> 4) & 3) {
        q = opaque(k == 0 ? 0x3ffc2f0u : k == 1 ? 0x3fffbffu : k < 10 ? 0x3ffffffu : 0u);
        one = opaque(k == 0 ? 1u : 0u);
        ge3 = mask_if(k >= 3);
        eq15 = mask_if(k == 15);
        ge14 = mask_if(k >= 14);
        lt10 = mask_if(k < 10);
        lt9 = mask_if(k < 9);
        keep9 = opaque(k < 9 ? M26 : 0xffffffffu);
        r0 = mask_if(row == 0);
        r1 = mask_if(row == 1);
        r2 = mask_if(row == 2);
    }
};
// m ? a : b, bitwise (v_bfi_b32)
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
__device__ __forceinline__ uint64_t bsel64(uint32_t m, uint64_t a, uint64_t b) {
    const uint64_t mm = (static_cast<uint64_t>(m) << 32) | m;
    return (a & mm) | (b & ~mm);
}

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
    return static_cast<uint64_t>(a) * b + c;
}
__device__ __forceinline__ uint32_t hi26(uint64_t x) {  // bits 26..57 of x
    return __builtin_amdgcn_alignbit(static_cast<uint32_t>(x >> 32), static_cast<uint32_t>(x), 26);
}

// the 19 columns (lo: lanes 0..15 = columns 0..15, hi: lanes 0..2 = columns 16..18, each < 2^63.4)
// -> a reduced element (see the header)
__device__ __forceinline__ uint32_t reduce(uint64_t lo, uint64_t hi, const Lane& L) {
    // round 1: column = l + cA 2^26 + cB 2^52 (cB < 2^11.4); cA goes one lane up, cB two
    const uint32_t l = static_cast<uint32_t>(lo) & M26, cA = hi26(lo) & M26, cB = static_cast<uint32_t>(lo >> 52);
    const uint32_t lh = static_cast<uint32_t>(hi) & M26, hA = hi26(hi) & M26, hB = static_cast<uint32_t>(hi >> 52);
    const uint32_t v = l + shr<1>(cA) + shr<2>(cB);  // columns 0..15, < 2^27.01
    // columns 16..20: lane 0 takes column 15's cA and column 14's cB, lane 1 column 15's cB (the lane
    // choice masks the DPP SOURCE: every DPP move runs on the whole row)
    const uint32_t x1 = shr<1>(hA) + ror<1>(cA & L.eq15);
    const uint32_t x2 = shr<2>(hB) + ror<2>(cB & L.ge14);
    const uint32_t w = lh + x1 + x2;  // lanes 0..4 = columns 16..20
    // fold: H_j = column 10 + j (lanes 0..10), into lane j (* R0) and lane j + 1 (* 2^10)
    const uint32_t H = shl<10>(v) + shr<6>(w);
    const uint32_t Hs = shr<1>(H);
    const uint64_t r = mad(H, R0, v & L.lt10) + (static_cast<uint64_t>(Hs) << 10);  // lanes 0..9 < 2^41.1; 10, 11 = columns 10, 11
    // round 3
    const uint32_t c3 = hi26(r);  // < 2^15.1
    const uint32_t u = (static_cast<uint32_t>(r) & M26) + shr<1>(c3);  // lanes 10, 11: columns 10, 11 (< 2^26.1, < 2^19.5)
    // fold columns 10, 11 into lanes 0..2
    const uint32_t G = shl<10>(u);
    const uint64_t t = mad(G, R0, u & L.lt10) + (static_cast<uint64_t>(shr<1>(G)) << 10);  // lane 0 < 2^40, lanes 1, 2 < 2^36
    // last carry: lanes 0..8 carry one lane up, lane 9 keeps its value (< 2^26 + 2^15.1)
    const uint32_t c5 = hi26(t) & L.lt9;
    return (static_cast<uint32_t>(t) & L.keep9) + shr<1>(c5);
}

// the product's 19 columns of a * b (both spread over the row, magnitudes <= 16): lo = columns 0..15 on
// lanes 0..15, hi = columns 16..18 on lanes 0..2.  Two accumulators (even / odd steps) halve the
// dependent chain of 64-bit multiply-adds.
__device__ __forceinline__ void conv(uint32_t a, uint32_t b, const Lane& L, uint64_t& lo, uint64_t& hi) {
    uint32_t t1 = ror<1>(b);
    uint64_t e = mad(bcast<0>(a), b, 0), o = mad(bcast<1>(a), t1, 0);
    uint32_t t2 = ror<2>(b);
    t1 = ror<2>(t1);
    e = mad(bcast<2>(a), t2, e);
    o = mad(bcast<3>(a), t1, o);
    t2 = ror<2>(t2);
    t1 = ror<2>(t1);
    e = mad(bcast<4>(a), t2, e);
    o = mad(bcast<5>(a), t1, o);
    t2 = ror<2>(t2);
    t1 = ror<2>(t1);
    e = mad(bcast<6>(a), t2, e);
    // steps 7..9: on lanes 0..2 the rotated sources are b_(16 + k - i), i.e. columns 16 + k
    t2 = ror<2>(t2);
    uint64_t we = mad(bcast<8>(a), t2, 0), wo = mad(bcast<7>(a), t1, 0);
    t1 = ror<2>(t1);
    wo = mad(bcast<9>(a), t1, wo);
    const uint64_t w = we + wo;
    lo = e + o + bsel64(L.ge3, w, 0);
    hi = bsel64(L.ge3, 0, w);
}
// r = a * b in secp256k1's field (magnitudes <= 16 -> 1)
__device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b, const Lane& L) {
    uint64_t lo, hi;
    conv(a, b, L, lo, hi);
    return reduce(lo, hi, L);
}

__device__ __forceinline__ uint32_t sqr(uint32_t a, const Lane& L) { return mul(a, a, L); }

__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
template <int K>
__device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b, const Lane& L) { return a + (K * L.q - b); }
template <int K>
__device__ __forceinline__ uint32_t neg(uint32_t a, const Lane& L) { return K * L.q - a; }
template <int C>
__device__ __forceinline__ uint32_t mul_int(uint32_t a) { return a * C; }

// ------------------------------------------------------------------ SM2's field on the rows
// p = 2^256 - 2^224 - 2^96 + 2^64 - 1 has no small 2^260 residue (2^260 = 2^228 + 2^100 - 2^68 + 2^4 mod
// p: folding by it alone would take eight rounds), so the high columns H_j (weight 2^(26 (10 + j)),
// j = 0..10) fold through their FULL residues M_j = 2^(26 (10 + j)) mod p: lane k adds
// sum_j H_j M_j[k] -- eleven broadcasts and multiply-adds, each M_j[k] < 2^26 a per-lane constant, the
// sum < 2^56.5; one parallel carry; then the carries into lanes 10, 11 (weights 2^260, 2^286: M_0 and
// M_1 are < 2^229 and < 2^255) and lane 9's bits from 2^256 (D = 2^256 mod p) fold once more, which
// leaves a value < 2^257, and two carry rounds bring every limb under B.  Same magnitude contracts as
// the secp256k1 field; sub<K> adds K Q2 with Q2 = 16 p in digits within 2^-4 of 2^26, so K Q2 >= b limb
// by limb for b.m <= K - 1 up to K = 15.  Checked on the GPU by tools/rowbench.hip against a host
// reference, and in Python (every bound above) at magnitude 16.
// 2^(26 (10 + j)) mod p for j = 0..10, D = 2^256 mod p and Q2 = 16 p (digit 2 raised by 2^26, digit 3
// lowered by 1, so every digit is within 2^-4 of 2^26), radix-2^26 digits per lane (lanes 10..15: 0)
__device__ __constant__ static const uint32_t kSm2RowM[11][16] = {
    {0x10u, 0x0u, 0x3ff0000u, 0x3fffffu, 0x0u, 0x0u, 0x0u, 0x0u, 0x100000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x0u, 0x10u, 0x0u, 0x3ff0000u, 0x3fffffu, 0x0u, 0x0u, 0x0u, 0x0u, 0x100000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x1000000u, 0x0u, 0x10u, 0x3fffc00u, 0x3ffffffu, 0x3fffffu, 0x0u, 0x0u, 0x0u, 0x4000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x40000u, 0x1000000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x400000u, 0x0u, 0x0u, 0x100u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x1000u, 0x40000u, 0x0u, 0x0u, 0x10u, 0x0u, 0x0u, 0x400000u, 0x0u, 0x4u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x40u, 0x1000u, 0x0u, 0x1000000u, 0x0u, 0x10u, 0x0u, 0x0u, 0x800000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x2u, 0x40u, 0x3fff000u, 0x7ffffu, 0x1000000u, 0x0u, 0x10u, 0x0u, 0x20000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x0u, 0x2u, 0x40u, 0x3fff000u, 0x7ffffu, 0x1000000u, 0x0u, 0x10u, 0x0u, 0x20000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x200000u, 0x0u, 0x2u, 0x3ffffc0u, 0xfffu, 0x80000u, 0x1000000u, 0x0u, 0x10u, 0x800u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x8000u, 0x200000u, 0x0u, 0x0u, 0x40u, 0x1000u, 0x80000u, 0x1000000u, 0x0u, 0x30u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
    {0x300u, 0x8000u, 0x3f00000u, 0x3ffffffu, 0x2u, 0x40u, 0x1000u, 0x80000u, 0x0u, 0x1u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u},
};
__device__ __constant__ static const uint32_t kSm2RowD[16] = {0x1u, 0x0u, 0x3fff000u, 0x3ffffu, 0x0u, 0x0u, 0x0u, 0x0u, 0x10000u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u};
__device__ __constant__ static const uint32_t kSm2RowQ[16] = {0x3fffff0u, 0x3ffffffu, 0x400ffffu, 0x3bfffffu, 0x3ffffffu, 0x3ffffffu, 0x3ffffffu, 0x3ffffffu, 0x3efffffu, 0x3ffffffu, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u};

struct Sm2Lane {
    uint32_t q, d, mask9;  // Q2 and D digits, mask9: all ones on lanes 0..8, 2^22 - 1 on lane 9, 0 above
    uint32_t m[11];
    __device__ __forceinline__ explicit Sm2Lane(const Lane& L) {
        q = kSm2RowQ[L.k];
        d = kSm2RowD[L.k];
#pragma unroll
        for (int j = 0; j < 11; ++j) m[j] = kSm2RowM[j][L.k];
        mask9 = opaque(L.k < 9 ? 0xffffffffu : L.k == 9 ? 0x3fffffu : 0u);
    }
};

template <int J>
__device__ __forceinline__ uint64_t fold_col(uint32_t H, const Sm2Lane& C, uint64_t r) {
    return mad(bcast<J>(H), C.m[J], r);
}

__device__ __forceinline__ uint32_t reduce_sm2(uint64_t lo, uint64_t hi, const Lane& L, const Sm2Lane& C) {
    // round 1 (as reduce): columns 0..15 in v, 16..20 in w
    const uint32_t l = static_cast<uint32_t>(lo) & M26, cA = hi26(lo) & M26, cB = static_cast<uint32_t>(lo >> 52);
    const uint32_t lh = static_cast<uint32_t>(hi) & M26, hA = hi26(hi) & M26, hB = static_cast<uint32_t>(hi >> 52);
    const uint32_t v = l + shr<1>(cA) + shr<2>(cB);
    const uint32_t x1 = shr<1>(hA) + ror<1>(cA & L.eq15);
    const uint32_t x2 = shr<2>(hB) + ror<2>(cB & L.ge14);
    const uint32_t w = lh + x1 + x2;
    const uint32_t H = shl<10>(v) + shr<6>(w);  // lanes 0..10: H_j = column 10 + j (< 2^27.01)
    // pass 1: r_k = v_k + sum_j H_j M_j[k]  (< 2^56.5, lanes 0..9)
    // (three accumulators: the multiply-adds' dependent chain is four long instead of eleven)
    uint64_t ra = fold_col<0>(H, C, v & L.lt10), rb = fold_col<1>(H, C, 0), rc = fold_col<2>(H, C, 0);
    ra = fold_col<3>(H, C, ra);
    rb = fold_col<4>(H, C, rb);
    rc = fold_col<5>(H, C, rc);
    ra = fold_col<6>(H, C, ra);
    rb = fold_col<7>(H, C, rb);
    rc = fold_col<8>(H, C, rc);
    ra = fold_col<9>(H, C, ra);
    rb = fold_col<10>(H, C, rb);
    const uint64_t r = ra + rb + rc;
    const uint32_t u = (static_cast<uint32_t>(r) & M26) + shr<1>(hi26(r) & M26) + shr<2>(static_cast<uint32_t>(r >> 52));
    // pass 2: lanes 10, 11 by M_0, M_1; lane 9's bits from 2^256 by D  (< 2^52.1)
    const uint64_t t = mad(bcast<10>(u), C.m[0], u & C.mask9) + mad(bcast<11>(u), C.m[1], 0) +
                       mad(bcast<9>(u) >> 22, C.d, 0);
    // round A (lane 9 stays < 2^24.8, so nothing leaves it), round B (lanes 0..8 carry)
    const uint32_t ua = (static_cast<uint32_t>(t) & M26) + shr<1>(hi26(t) & M26) + shr<2>(static_cast<uint32_t>(t >> 52));
    return ((ua & L.keep9) + shr<1>((ua >> 26) & L.lt9)) & L.lt10;
}
__device__ __forceinline__ uint32_t mul_sm2(uint32_t a, uint32_t b, const Lane& L, const Sm2Lane& C) {
    uint64_t lo, hi;
    conv(a, b, L, lo, hi);
    return reduce_sm2(lo, hi, L, C);
}
template <int K>
__device__ __forceinline__ uint32_t sub_sm2(uint32_t a, uint32_t b, const Sm2Lane& C) { return a + (K * C.q - b); }
template <int K>
__device__ __forceinline__ uint32_t neg_sm2(uint32_t a, const Sm2Lane& C) { return K * C.q - a; }

// every row receives every row's value: .v[j] = row j's (v_permlane16_swap then v_permlane32_swap)
struct Rows4 {
    uint32_t v[4];
};
__device__ __forceinline__ Rows4 gather4(uint32_t p) {
    const auto a = __builtin_amdgcn_permlane16_swap(p, p, false, false);        // [p0 p0 p2 p2], [p1 p1 p3 p3]
    const auto b = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);  // [p0 p0 p0 p0], [p2 p2 p2 p2]
    const auto c = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);  // [p1 p1 p1 p1], [p3 p3 p3 p3]
    return Rows4{{b[0], c[0], b[1], c[1]}};
}
// row 0's and row 1's values on every row
__device__ __forceinline__ void gather01(uint32_t p, uint32_t& p0, uint32_t& p1) {
    const auto a = __builtin_amdgcn_permlane16_swap(p, p, false, false);
    p0 = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false)[0];
    p1 = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false)[0];
}
// row 0's value on every row
__device__ __forceinline__ uint32_t gather0(uint32_t p) {
    const auto a = __builtin_amdgcn_permlane16_swap(p, p, false, false);
    return __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false)[0];
}
// per-row operand choice
__device__ __forceinline__ uint32_t sel4(const Lane& L, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3) {
    return bsel(L.r0, r0, bsel(L.r1, r1, bsel(L.r2, r2, r3)));
}

}  // namespace frow
}  // namespace bcosgpu
