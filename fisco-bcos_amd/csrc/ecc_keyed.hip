// ecc_keyed.hip -- signature verification against REGISTERED public keys: the sealer path.
//
// SignatureCrypto::verify(pub, hash, sig) is called with a small, fixed set of keys on the block-check
// path: BlockValidator::checkSignatureList verifies one signature per sealer of the block against the
// consensus node list's keys (bcos-pbft/.../BlockValidator.cpp:141-182), PBFTCacheProcessor::
// checkPrecommitWeight likewise (PBFTCacheProcessor.cpp:795-821), both through Secp256k1Crypto.cpp:51-63 /
// SM2Crypto.cpp:66-79.  With the key known in advance, its variable-base multiplication needs no
// doublings at verify time: the engine keeps an 8-bit comb table per key (32 windows x 256 affine
// multiples b 2^(8i) P, 512 KiB of HBM, built once by key_table_kernel), so u2 P (secp256k1) / t P (SM2)
// is 32 table lookups, like u1 G / s G over G's 16-bit comb (16 lookups).
//
// The verify kernel spends 16 lanes (one DPP row) on each signature, 4 signatures per wave:
//   - every lane of the 16 runs the scalar work (range checks, s^-1 mod n and u1, u2 for secp256k1;
//     t = r + s and e = SM3(Z_A || h) with Z_A cached per key for SM2) -- in lockstep, so it costs the
//     same as on one lane;
//   - lane L sums its three table points (windows 2L, 2L+1 of the key's comb, window L of G's 16-bit
//     comb; the 8-bit G comb adds windows 2L, 2L+1 of it instead) with complete mixed additions;
//   - four levels of complete Jacobian additions reduce the 16 partial sums inside the row (partners
//     fetched with ds_bpermute), then the projective x-check (no inversion) gives the verdict.
// Critical path: secp256k1 ~ s^-1 + 3 madds + 4 adds, SM2 ~ 2 SM3 compressions + 3 madds + 4 adds --
// against 256 doublings per signature on the generic path.  Same decisions and verdicts as
// secp256k1_verify_lane26 / sm2_verify_rs26 (libsecp256k1 ecdsa_verify with low-S; sm2_do_verify), for
// every input: the additions are the complete ones (P = Q, P = -Q, infinity), since a key's owner can
// pick u1, u2 so that two partial sums coincide.
//
// Host side: a per-(device, suite) cache of key tables, filled by bcosgpu_register_keys (the node's
// consensus list) and by promotion of keys named in three verify calls (counted once per call; SM2
// recover -- admission, the sender's own key -- never promotes; at most 16 keys a build, one build in
// flight, built asynchronously and published when done, in at most half the capacity); never evicted while the process runs (bcosgpu_clear_keys drains the device first), so a
// table is never rewritten under a launch that reads it.  Slot ids carry the cache generation: an id from
// before a clear fails in the kernel instead of naming whichever key now has its index.  The coalesced
// host-pointer verify calls take this path when every key of the batch is cached.
#include <algorithm>
#include <array>
#include <atomic>
#include <unordered_map>
#include <unordered_set>
#include "ecc_device.h"

namespace bcosgpu {

// per key slot: a 64-word header, then the comb table [32 windows][256 entries][x[8] y[8]]
//   header: [0..7] x, [8..15] y (canonical, plain), [16..23] Z_A (SM2: SM3 state words), [24..28] the
//   address right160(H(pub)) as the kernels store it (Keccak256 secp256k1 / SM3 SM2), [32] 1 = valid key
//   (coordinates < p, on the curve)
static constexpr size_t kKeyHdrWords = 64;
static constexpr size_t kKeySlotWords = kKeyHdrWords + kTabWords;
static constexpr int kKeyEntriesPerKey = kCombWindows * kCombEntries;  // 8192 table lanes per key

// SM2 Z_A = SM3(ENTL || ID || a || b || xG || yG || xA || yA): the key-independent 128-byte prefix is the
// constant midstate kZaMid, then two blocks (as sm2_e's first half)
__device__ __forceinline__ void sm2_za(uint32_t V[8], const uint32_t X[8], const uint32_t Y[8]) {
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) V[i] = kZaMid[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) W[j] = kZaW32[j];
    W[4] = kZaC36 | (X[0] >> 16);
#pragma unroll
    for (int j = 1; j < 8; ++j) W[4 + j] = (X[j - 1] << 16) | (X[j] >> 16);
    W[12] = (X[7] << 16) | (Y[0] >> 16);
#pragma unroll
    for (int j = 1; j < 4; ++j) W[12 + j] = (Y[j - 1] << 16) | (Y[j] >> 16);
    sm3_compress(V, W);
#pragma unroll
    for (int j = 0; j < 4; ++j) W[j] = (Y[j + 3] << 16) | (Y[j + 4] >> 16);
    W[4] = (Y[7] << 16) | 0x8000u;
#pragma unroll
    for (int j = 5; j < 15; ++j) W[j] = 0;
    W[15] = 210u * 8u;
    sm3_compress(V, W);
}

// e = SM3(Z_A || hash) (sm2_e's second half)
__device__ __forceinline__ void sm2_e_from_za(fe& e, const uint32_t* za, const fe& hash_be) {
    uint32_t V[8], W[16];
    sm3_init(V);
#pragma unroll
    for (int j = 0; j < 8; ++j) W[j] = za[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) W[8 + j] = hash_be.v[7 - j];
    sm3_compress(V, W);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = 0;
    W[0] = 0x80000000u;
    W[15] = 512u;
    sm3_compress(V, W);
#pragma unroll
    for (int i = 0; i < 8; ++i) e.v[i] = V[7 - i];
}

// ------------------------------------------------------------------ table build
// Two launches.  BASES: lane (key k, window i) computes the window's base 2^(8i) P (8i doublings, one
// inversion to affine) into `base`; then lane (key k, window i, entry b) computes b 2^(8i) P by an 8-bit
// double-and-add of that base and one inversion.  The chain of 8i doublings runs once per window instead
// of once per entry (the build's work ~5x smaller, its latency one short launch longer), so a promotion
// build beside live batches takes less of the GPU from them.  secp256k1 entries are canonical plain words; SM2 entries canonical words of the
// R' = 2^286 Montgomery form (the layout of the fp26 G tables, tables_sm2_26).  Entry 0 holds 1 2^(8i) P
// (a valid point the kernels never select).  An invalid key (coordinates >= p or off the curve) gets
// G's multiples and valid = 0, which makes every verify against it fail, as the reference's does.
template <int SUITE, bool BASES>
__global__ __launch_bounds__(256) void key_table_kernel(uint32_t* __restrict__ arena, const int32_t* __restrict__ slots,
                                                        const uint8_t* __restrict__ pubs, uint32_t nkeys,
                                                        uint32_t* __restrict__ base) {
    const uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    constexpr uint64_t per = BASES ? kCombWindows : kKeyEntriesPerKey;
    if (idx >= static_cast<uint64_t>(nkeys) * per) return;
    const uint32_t k = static_cast<uint32_t>(idx / per);
    const uint32_t ent = BASES ? static_cast<uint32_t>(idx % per) * kCombEntries + 1u : static_cast<uint32_t>(idx % per);
    const int win = static_cast<int>(ent / kCombEntries);
    uint32_t b = ent % kCombEntries;
    if (b == 0) b = 1;
    uint32_t* slot = arena + static_cast<size_t>(slots[k]) * kKeySlotWords;
    uint32_t* bp = base + (static_cast<size_t>(k) * kCombWindows + win) * 16;  // the window's base (affine)
    uint32_t* out = BASES ? bp : slot + kKeyHdrWords + static_cast<size_t>(ent) * 16;
    ByteReader rp(pubs + 64ull * k, 64);
    uint32_t w[8], X[8], Y[8];
    fe px, py;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        X[q] = bswap32(rp.word(q));
        Y[q] = bswap32(rp.word(8 + q));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = rp.word(q);
    fe_from_be_words(px, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = rp.word(8 + q);
    fe_from_be_words(py, w);
    if constexpr (SUITE == BCOSGPU_SUITE_SECP256K1) {
        bool valid = fe_lt_k(px, FieldK1::P) && fe_lt_k(py, FieldK1::P);
        Aff26 P;
        fe26_from_fe(P.x, px);
        fe26_from_fe(P.y, py);
        {
            fe26 l, rr, t, seven;
            fe26_sqr(l, P.y);
            fe26_sqr(t, P.x);
            fe26_mul(rr, t, P.x);
            fe26_set_small(seven, 7u);
            fe26_add(rr, rr, seven);
            fe26_sub<3>(l, l, rr);
            valid = valid && fe26_is_zero(l);
        }
        if (!BASES) {  // the window's base, G's multiple for an invalid key
            fe bx, by;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                bx.v[q] = bp[q];
                by.v[q] = bp[8 + q];
            }
            fe26_from_fe(P.x, bx);
            fe26_from_fe(P.y, by);
        } else if (!valid) {
            fe26_const(P.x, kK1Gx);
            fe26_const(P.y, kK1Gy);
        }
        Jac26 acc, S;
        CurveK1x::set_inf(acc);
#pragma unroll 1
        for (int bit = 7; bit >= 0; --bit) {
            CurveK1x::dbl(acc, acc);
            CurveK1x::madd(S, acc, P);
            CurveK1x::cmov(acc, S, ((b >> bit) & 1u) != 0u);
        }
        if (BASES) {
#pragma unroll 1
            for (int d = 0; d < 8 * win; ++d) CurveK1x::dbl(acc, acc);
        }
        fe z, zi;
        fe26_to_fe(z, acc.Z);
        modinv_safegcd(zi, z, kMod30K1P);
        fe26 Zi, Zi2, Zi3, ax, ay;
        fe26_from_fe(Zi, zi);
        fe26_sqr(Zi2, Zi);
        fe26_mul(Zi3, Zi2, Zi);
        fe26_mul(ax, acc.X, Zi2);
        fe26_mul(ay, acc.Y, Zi3);
        fe x, y;
        fe26_to_fe(x, ax);
        fe26_to_fe(y, ay);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            out[q] = x.v[q];
            out[8 + q] = y.v[q];
        }
        if (!BASES && ent == 0) {
            uint32_t a[5];
            keccak_address(a, px, py);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                slot[q] = px.v[q];
                slot[8 + q] = py.v[q];
                slot[16 + q] = 0;
            }
#pragma unroll
            for (int q = 0; q < 5; ++q) slot[24 + q] = a[q];
            slot[32] = valid ? 1u : 0u;
        }
    } else {
        bool valid = fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
        AffP26 P;
        fp26_from_plain(P.x, px);
        fp26_from_plain(P.y, py);
        valid = valid && sm2_on_curve26(P);
        if (!BASES) {  // the window's base, G's multiple for an invalid key
            fe bx, by;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                bx.v[q] = bp[q];
                by.v[q] = bp[8 + q];
            }
            fp26_from_fe(P.x, bx);
            fp26_from_fe(P.y, by);
        } else if (!valid) {
            fe gx, gy;
            fe_set(gx, kSM2Gx);  // Montgomery (R = 2^256) form: back to plain first
            fe_set(gy, kSM2Gy);
            FieldP2::to_plain(gx, gx);
            FieldP2::to_plain(gy, gy);
            fp26_from_plain(P.x, gx);
            fp26_from_plain(P.y, gy);
        }
        JacP26 acc, S;
        CurveSM2x::set_inf(acc);
#pragma unroll 1
        for (int bit = 7; bit >= 0; --bit) {
            CurveSM2x::dbl(acc, acc);
            CurveSM2x::madd(S, acc, P);
            CurveSM2x::cmov(acc, S, ((b >> bit) & 1u) != 0u);
        }
        if (BASES) {
#pragma unroll 1
            for (int d = 0; d < 8 * win; ++d) CurveSM2x::dbl(acc, acc);
        }
        fp26 zi, zi2, zi3, ax, ay;
        fp26_inv(zi, acc.Z);
        fp26_sqr(zi2, zi);
        fp26_mul(zi3, zi2, zi);
        fp26_mul(ax, acc.X, zi2);
        fp26_mul(ay, acc.Y, zi3);
        fe x, y;
        fp26_to_fe(x, ax);
        fp26_to_fe(y, ay);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            out[q] = x.v[q];
            out[8 + q] = y.v[q];
        }
        if (!BASES && ent == 0) {
            uint32_t V[8], a[5];
            sm2_za(V, X, Y);
            sm3_address(a, px, py);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                slot[q] = px.v[q];
                slot[8 + q] = py.v[q];
                slot[16 + q] = V[q];
            }
#pragma unroll
            for (int q = 0; q < 5; ++q) slot[24 + q] = a[q];
            slot[32] = valid ? 1u : 0u;
        }
    }
}

// ------------------------------------------------------------------ verify
// the 16-lane row's partial sums -> lane 0 (lanes of a row are 16-aligned: __shfl_down with width 16)
template <class J, int LIMBS>
__device__ __forceinline__ void shfl_down_point(J& o, const J& a, int off) {
#pragma unroll
    for (int q = 0; q < LIMBS; ++q) {
        o.X.v[q] = __shfl_down(a.X.v[q], off, 16);
        o.Y.v[q] = __shfl_down(a.Y.v[q], off, 16);
        o.Z.v[q] = __shfl_down(a.Z.v[q], off, 16);
    }
    o.inf = __shfl_down(static_cast<int>(a.inf), off, 16) != 0;
}

// word q of k for a lane-varying q, by selects (a dynamic index would put k in scratch memory)
__device__ __forceinline__ uint32_t word_of(const fe& k, int q) {
    uint32_t w = k.v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) w = q == j ? k.v[j] : w;
    return w;
}
__device__ __forceinline__ uint32_t byte_of(const fe& k, int j) { return (word_of(k, j >> 2) >> ((j & 3) * 8)) & 0xffu; }
__device__ __forceinline__ uint32_t half_of(const fe& k, int j) { return (word_of(k, j >> 1) >> ((j & 1) * 16)) & 0xffffu; }

// acc += the comb entry at tab when its digit d != 0 (complete mixed addition)
__device__ __forceinline__ void keyed_add_entry(Jac26& acc, const uint32_t* tab, uint32_t d) {
    Aff26 T;
    load_aff26(T, tab);
    Jac26 S;
    CurveK1x::madd(S, acc, T);
    CurveK1x::cmov(acc, S, d != 0u);
}
__device__ __forceinline__ void keyed_add_entry(JacP26& acc, const uint32_t* tab, uint32_t d) {
    AffP26 T;
    load_affp26(T, tab);
    JacP26 S;
    CurveSM2x::madd(S, acc, T);
    CurveSM2x::cmov(acc, S, d != 0u);
}

// ok[i] = SignatureCrypto::verify(key of slot[i], hash[i], sig[i]); addr (SM2 tx admission: the verified
// key's SM3 address) may be null.  One 64-thread workgroup = 4 signatures.
template <int SUITE>
__global__ __launch_bounds__(64) void sig_verify_keyed_kernel(const uint32_t* __restrict__ arena, uint32_t cap,
                                                              uint32_t gen15, const int32_t* __restrict__ slots,
                                                              const uint8_t* __restrict__ hash,
                                                              const uint8_t* __restrict__ sig, uint32_t stride,
                                                              uint64_t n, const uint32_t* __restrict__ gtab, int gbits,
                                                              uint8_t* __restrict__ okout, uint8_t* __restrict__ addr) {
    const uint32_t lane = threadIdx.x;
    const int L = static_cast<int>(lane & 15u);
    const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * 4u + (lane >> 4);
    const bool live = i0 < n;
    const uint64_t i = live ? i0 : n - 1;  // a spare row re-runs the last signature (nothing stored)
    // a slot id is (generation << 16) | index (keyed_slots): an id handed out before a bcosgpu_clear_keys
    // names an old generation and fails here, even once its index holds another key's table
    const int32_t sl = slots[i];
    const uint32_t idx = static_cast<uint32_t>(sl) & 0xFFFFu;
    const bool slot_ok = sl >= 0 && (static_cast<uint32_t>(sl) >> 16) == gen15 && idx < cap;
    const uint32_t* key = arena + static_cast<size_t>(slot_ok ? idx : 0) * kKeySlotWords;
    const uint32_t* ktab = key + kKeyHdrWords;
    fe h;
    load_be256(h, hash + 32 * i);
    ByteReader rs(sig + static_cast<uint64_t>(stride) * i, 64);
    uint32_t w[8];
    fe r, s;
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = rs.word(q);
    fe_from_be_words(r, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = rs.word(8 + q);
    fe_from_be_words(s, w);
    bool ok = slot_ok && key[32] == 1u;
    bool match = false;
    if constexpr (SUITE == BCOSGPU_SUITE_SECP256K1) {
        ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN1::M) && fe_lt_k(s, kN1HalfPlus);
        fe e;
        fe_copy(e, h);
        reduce_once(e, ParamN1::M);
        fe ss = s;
        if (!ok) {
            fe_zero(ss);
            ss.v[0] = 1;
        }
        fe sm, sinv, u1, u2;
        FieldN1::from_plain(sm, ss);
        FieldInv<FieldN1>::inv_pipe(sinv, sm);
        FieldN1::mul(u1, e, sinv);
        FieldN1::mul(u2, r, sinv);
        Jac26 acc;
        CurveK1x::set_inf(acc);
        const uint32_t b0 = byte_of(u2, 2 * L), b1 = byte_of(u2, 2 * L + 1);
        keyed_add_entry(acc, ktab + (static_cast<size_t>(2 * L) * kCombEntries + b0) * 16, b0);
        keyed_add_entry(acc, ktab + (static_cast<size_t>(2 * L + 1) * kCombEntries + b1) * 16, b1);
        if (gbits == kWideBits) {
            const uint32_t g = half_of(u1, L);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(L) * kWideEntries + g) * 16, g);
        } else {
            const uint32_t g0 = byte_of(u1, 2 * L), g1 = byte_of(u1, 2 * L + 1);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(2 * L) * kCombEntries + g0) * 16, g0);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(2 * L + 1) * kCombEntries + g1) * 16, g1);
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            Jac26 o;
            shfl_down_point<Jac26, 10>(o, acc, off);
            CurveK1x::add(acc, acc, o);
        }
        ok = ok && !acc.inf;
        fe26 z2, rhs, R, d;
        fe26_sqr(z2, acc.Z);
        fe26_from_fe(R, r);
        fe26_mul(rhs, R, z2);
        fe26_sub<10>(d, rhs, acc.X);  // acc.X <= 9: an addition may pass a mixed sum through
        match = fe26_is_zero(d);
        fe r2;
        const uint32_t carry = fe_add_k(r2, r, ParamN1::M);
        if (carry == 0u && fe_lt_k(r2, FieldK1::P)) {
            fe26_from_fe(R, r2);
            fe26_mul(rhs, R, z2);
            fe26_sub<10>(d, rhs, acc.X);
            match = match || fe26_is_zero(d);
        }
    } else {
        ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
        fe t;
        FieldN2::add(t, r, s);
        ok = ok && !fe_is_zero_raw(t);
        fe e;
        sm2_e_from_za(e, key + 16, h);
        reduce_once(e, ParamN2::M);
        JacP26 acc;
        CurveSM2x::set_inf(acc);
        const uint32_t b0 = byte_of(t, 2 * L), b1 = byte_of(t, 2 * L + 1);
        keyed_add_entry(acc, ktab + (static_cast<size_t>(2 * L) * kCombEntries + b0) * 16, b0);
        keyed_add_entry(acc, ktab + (static_cast<size_t>(2 * L + 1) * kCombEntries + b1) * 16, b1);
        if (gbits == kWideBits) {
            const uint32_t g = half_of(s, L);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(L) * kWideEntries + g) * 16, g);
        } else {
            const uint32_t g0 = byte_of(s, 2 * L), g1 = byte_of(s, 2 * L + 1);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(2 * L) * kCombEntries + g0) * 16, g0);
            keyed_add_entry(acc, gtab + (static_cast<size_t>(2 * L + 1) * kCombEntries + g1) * 16, g1);
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            JacP26 o;
            shfl_down_point<JacP26, 10>(o, acc, off);
            CurveSM2x::add(acc, acc, o);
        }
        ok = ok && !acc.inf;
        // x1 = X / Z^2 must be congruent to r - e (mod n): x1 = c or c + n (when c + n < p)
        fe c, c2;
        FieldN2::sub(c, r, e);
        fp26 z2, cm, rhs, dlt;
        fp26_sqr(z2, acc.Z);
        fp26_from_plain(cm, c);
        fp26_mul(rhs, cm, z2);
        fp26_sub<13>(dlt, rhs, acc.X);
        match = fp26_is_zero(dlt);
        const uint32_t carry = fe_add_k(c2, c, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            fp26_from_plain(cm, c2);
            fp26_mul(rhs, cm, z2);
            fp26_sub<13>(dlt, rhs, acc.X);
            match = match || fp26_is_zero(dlt);
        }
    }
    ok = ok && match;
    if (live && L == 0) {
        okout[i] = ok ? 1 : 0;
        if (addr) {
            uint32_t* a = reinterpret_cast<uint32_t*>(addr + 20 * i);
#pragma unroll
            for (int q = 0; q < 5; ++q) a[q] = ok ? key[24 + q] : 0u;
        }
    }
}

// ------------------------------------------------------------------ host: the key cache
namespace {

using Key64 = std::array<uint8_t, 64>;
struct Key64Hash {
    size_t operator()(const Key64& k) const {
        uint64_t h;
        std::memcpy(&h, k.data() + 24, 8);  // low bits of x: uniformly distributed for valid keys
        uint64_t g;
        std::memcpy(&g, k.data() + 56, 8);
        return static_cast<size_t>(h ^ (g * 0x9E3779B97F4A7C15ull));
    }
};

struct KeyCache {
    std::mutex mu;
    std::mutex init_mu;              // prepare_promotion
    std::atomic<bool> ready{false};  // ... has run
    uint32_t* arena = nullptr;
    int cap = 0;
    bool alloc_failed = false;
    std::unordered_map<Key64, int32_t, Key64Hash> slot_of;  // published: table built
    std::unordered_map<Key64, int32_t, Key64Hash> pending;  // promoted, table being built (async)
    int32_t next = 0;  // arena indices handed out this generation (published, pending, failed builds)
    // the one promotion build in flight: on its own lowest-priority stream, published (slot_of) by the
    // first cache call after its event completes (poll_build)
    bool building = false;
    uint64_t build_gen = 0;
    hipStream_t build_stream = nullptr;
    hipEvent_t build_done = nullptr;
    std::vector<Key64> build_keys;
    std::vector<uint8_t> build_host;  // the build's upload source, alive until the build completes
    std::unordered_map<Key64, uint32_t, Key64Hash> seen;
    uint64_t hits = 0, misses = 0, builds = 0;
    int promoted = 0;  // slots taken by promotion: at most half the capacity, the rest stays for registrations
    int registered = 0;
    uint64_t gen = 0;  // bumped by keyed_clear: a slot looked up under another generation may name another key
    // the builds' key / slot upload buffer, grow-only: a build under mu costs its upload, the table kernel
    // and one stream sync, not a hipMalloc + hipFree (a hipFree can wait for the whole device)
    uint8_t* scratch = nullptr;
    size_t scratch_cap = 0;
};

std::mutex g_kc_mu;
KeyCache* g_kc[64][2] = {};  // never freed: no teardown races with the HIP runtime at exit

KeyCache* cache_of(int device, int suite) {
    std::lock_guard<std::mutex> g(g_kc_mu);
    KeyCache*& c = g_kc[device][suite];
    if (!c) c = new KeyCache();
    return c;
}

int capacity_env() {
    static const int cap = [] {
        const char* e = getenv("BCOSGPU_KEY_CACHE");  // keys per (device, suite); 512 KiB each
        const long v = e ? atol(e) : 256;
        return static_cast<int>(v < 0 ? 0 : v > 65536 ? 65536 : v);
    }();
    return cap;
}

// the 15-bit generation tag of public slot ids: id = (tag << 16) | index (capacity <= 65536 keys)
inline uint32_t gen_tag(uint64_t gen) { return static_cast<uint32_t>(gen & 0x7FFFu); }
inline int32_t slot_id(uint64_t gen, int32_t index) { return static_cast<int32_t>((gen_tag(gen) << 16) | uint32_t(index)); }

// tables built by one promotion build at most (keyed_slots: asynchronous, one in flight)
constexpr int kPromoteBuildsPerCall = 16;

int promote_after() {
    static const int k = [] {
        // calls that must see a key before it is cached (0 = never).  3: a sealer's key is cached by its
        // third block, while admission traffic over many distinct keys (each seen once or twice) does not
        // fill the cache with one-off keys
        const char* e = getenv("BCOSGPU_KEY_PROMOTE");
        return e ? atoi(e) : 3;
    }();
    return k;
}

// Under c.mu: the key arena, allocated on first use (capacity_env() tables).
void ensure_arena(KeyCache& c) {
    if (c.arena || c.alloc_failed) return;
    const int cap = capacity_env();
    if (cap > 0 && hipMalloc(&c.arena, static_cast<size_t>(cap) * kKeySlotWords * 4) == hipSuccess) {
        c.cap = cap;
    } else {
        (void)hipGetLastError();
        c.arena = nullptr;
        c.alloc_failed = true;
    }
}

// Under c.mu on the current device: build the tables of `keys` at arena indices `idx` on st -- with
// `async`, record c.build_done after it and return (c.build_host keeps the upload's source), else
// synchronise st.  One build uses c.scratch at a time: an async one is in flight only while c.building,
// and a synchronous one (registration) first waits for it (keyed_slots).
int build_tables(KeyCache& c, int suite, const std::vector<Key64>& keys, const std::vector<int32_t>& idx,
                 hipStream_t st, bool async) {
    const size_t kb = 64 * keys.size(), sb = 4 * idx.size();
    const size_t bo = (kb + sb + 255) & ~size_t{255}, bb = 64ull * kCombWindows * keys.size();  // window bases
    std::vector<uint8_t>& host = c.build_host;
    host.resize(kb + sb);
    for (size_t q = 0; q < keys.size(); ++q) std::memcpy(host.data() + 64 * q, keys[q].data(), 64);
    std::memcpy(host.data() + kb, idx.data(), sb);
    hipError_t e = hipSuccess;
    if (c.scratch_cap < bo + bb) {
        if (c.scratch) (void)hipFree(c.scratch);
        c.scratch = nullptr;
        c.scratch_cap = 0;
        const size_t want = std::max<size_t>(bo + bb, 256 + (64 * kCombWindows + 68) * 16);
        e = hipMalloc(reinterpret_cast<void**>(&c.scratch), want);
        if (e == hipSuccess) c.scratch_cap = want;
        else c.scratch = nullptr;
    }
    uint8_t* d = c.scratch;
    if (e == hipSuccess) e = hipMemcpyAsync(d, host.data(), kb + sb, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        const uint64_t nk = keys.size(), lanes1 = nk * kCombWindows, lanes2 = nk * kKeyEntriesPerKey;
        const dim3 g1(static_cast<unsigned>((lanes1 + 255) / 256)), g2(static_cast<unsigned>((lanes2 + 255) / 256));
        const int32_t* ds = reinterpret_cast<const int32_t*>(d + kb);
        uint32_t* db = reinterpret_cast<uint32_t*>(d + bo);
        if (suite == BCOSGPU_SUITE_SM2) {
            hipLaunchKernelGGL((key_table_kernel<BCOSGPU_SUITE_SM2, true>), g1, dim3(256), 0, st, c.arena, ds, d,
                               static_cast<uint32_t>(nk), db);
            hipLaunchKernelGGL((key_table_kernel<BCOSGPU_SUITE_SM2, false>), g2, dim3(256), 0, st, c.arena, ds, d,
                               static_cast<uint32_t>(nk), db);
        } else {
            hipLaunchKernelGGL((key_table_kernel<BCOSGPU_SUITE_SECP256K1, true>), g1, dim3(256), 0, st, c.arena, ds, d,
                               static_cast<uint32_t>(nk), db);
            hipLaunchKernelGGL((key_table_kernel<BCOSGPU_SUITE_SECP256K1, false>), g2, dim3(256), 0, st, c.arena, ds,
                               d, static_cast<uint32_t>(nk), db);
        }
        e = hipGetLastError();
        const hipError_t e2 = async ? hipEventRecord(c.build_done, st) : hipStreamSynchronize(st);
        if (e == hipSuccess) e = e2;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return BCOSGPU_E_HIP;
    }
    return 0;
}

// Outside c.mu, once per cache: what the first promotion needs -- the arena, the build stream and event,
// and the code object holding the table kernel (HIP loads it on first use, ~10 ms) -- so that no lookup
// waits behind these one-time costs.  Failures leave promotion off (build_stream null).
void prepare_promotion(KeyCache& c, int suite) {
    std::unique_lock<std::mutex> i(c.init_mu, std::try_to_lock);  // another caller preparing: skip, this
    if (!i.owns_lock() || c.ready.load(std::memory_order_acquire)) return;  // call does not promote
    bool need_arena;
    {
        std::lock_guard<std::mutex> g(c.mu);
        need_arena = !c.arena && !c.alloc_failed;
    }
    uint32_t* arena = nullptr;
    const int cap = capacity_env();
    if (need_arena && (cap <= 0 || hipMalloc(&arena, static_cast<size_t>(cap) * kKeySlotWords * 4) != hipSuccess)) {
        (void)hipGetLastError();
        arena = nullptr;
    }
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    hipFuncAttributes fa;
    int least = 0, greatest = 0;
    bool ok = hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
              hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least) == hipSuccess &&
              hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
    if (ok && suite == BCOSGPU_SUITE_SM2)
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&key_table_kernel<BCOSGPU_SUITE_SM2, true>)) == hipSuccess;
    else if (ok)
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&key_table_kernel<BCOSGPU_SUITE_SECP256K1, true>)) ==
             hipSuccess;
    if (!ok) (void)hipGetLastError();
    {
        std::lock_guard<std::mutex> g(c.mu);
        if (need_arena && !c.arena && arena) {
            c.arena = arena;
            c.cap = cap;
            arena = nullptr;
        } else if (need_arena && !c.arena) {
            c.alloc_failed = true;
        }
        if (ok) {
            c.build_stream = s;
            c.build_done = ev;
        }
    }
    if (arena) (void)hipFree(arena);  // a registration allocated the arena meanwhile
    c.ready.store(true, std::memory_order_release);
}

// Under c.mu: publish the promotion build in flight once it has completed (`wait`: block until then).
// A build from before a bcosgpu_clear_keys (another generation) or a failed one publishes nothing.
void poll_build(KeyCache& c, bool wait) {
    if (!c.building) return;
    hipError_t q = wait ? hipEventSynchronize(c.build_done) : hipEventQuery(c.build_done);
    if (q == hipErrorNotReady) return;
    c.building = false;
    const bool live = c.build_gen == c.gen;
    for (const Key64& k : c.build_keys) {
        auto it = live ? c.pending.find(k) : c.pending.end();
        if (it == c.pending.end()) continue;
        if (q == hipSuccess) {
            c.slot_of.emplace(k, it->second);
            c.seen.erase(k);
            ++c.builds;
            ++c.promoted;
        }
        c.pending.erase(it);
    }
    if (q != hipSuccess) (void)hipGetLastError();
    c.build_keys.clear();
}

}  // namespace

// Slot ids of n keys (pub i at pubs + pub_stride * i) on the current device; keys not cached are built
// when `force` (registration, synchronously: the ids returned name built tables), or -- when `promote` --
// once seen in promote_after() calls.  A key counts once per call however often it occurs in it, and only
// calls that name their keys explicitly promote (the sealer path: SignatureCrypto::verify(pub, ...));
// admission (SM2 recover, whose key is the sender's) only looks keys up.  A promotion build runs
// asynchronously on the cache's own lowest-priority stream, at most kPromoteBuildsPerCall keys and one
// build at a time: the batch that promotes a key, and every batch until its table is published, takes
// the generic kernels, so no caller waits for a build (a build is ~0.9 ms, latency-bound, whatever its
// key count: profiles/r06_tail_ab.json).  Ids carry the cache generation (slot_id).  Returns 0 and
// *all = every key has a slot, or < 0.
int keyed_slots(int suite, const uint8_t* pubs, size_t pub_stride, size_t n, int32_t* out, bool force, bool* all,
                hipStream_t st, uint64_t* gen, bool promote) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    *all = false;
    if (n == 0) {
        *all = true;
        return 0;
    }
    KeyCache& c = *cache_of(dev, suite == BCOSGPU_SUITE_SM2 ? 1 : 0);
    promote = promote && !force && promote_after() > 0;
    if (promote && !c.ready.load(std::memory_order_acquire)) prepare_promotion(c, suite);
    std::lock_guard<std::mutex> g(c.mu);
    poll_build(c, force);  // a registration reuses the scratch buffer: the build in flight finishes first
    if (gen) *gen = c.gen;
    promote = promote && c.build_stream && c.arena;
    if (!force && c.slot_of.empty() && !promote) return 0;
    std::vector<Key64> keys;      // tables this call builds ...
    std::vector<int32_t> idx;     // ... at these arena indices
    std::vector<size_t> want_at;  // (force) positions that take a key built by this call
    std::unordered_set<Key64, Key64Hash> first, counted;  // this call's keys being built / already counted
    bool every = true;
    for (size_t i = 0; i < n; ++i) {
        Key64 k;
        std::memcpy(k.data(), pubs + pub_stride * i, 64);
        auto it = c.slot_of.find(k);
        if (it != c.slot_of.end()) {
            out[i] = slot_id(c.gen, it->second);
            continue;
        }
        out[i] = -1;
        if (force && first.count(k)) {  // a repeat within this registration: it follows its first occurrence
            want_at.push_back(i);
            continue;
        }
        every = false;
        if (!force && (!promote || c.building || c.pending.count(k) || !counted.insert(k).second)) continue;
        bool build = force;
        if (!build && c.promoted + static_cast<int>(first.size()) < capacity_env() / 2 &&
            static_cast<int>(first.size()) < kPromoteBuildsPerCall) {
            if (c.seen.size() > (1u << 16)) c.seen.clear();  // a bounded sketch of recent keys
            build = ++c.seen[k] >= static_cast<uint32_t>(promote_after());
        }
        if (!build) continue;
        if (force) ensure_arena(c);
        if (!c.arena || c.next >= c.cap) continue;  // the cache is full: not cached
        first.insert(k);
        keys.push_back(k);
        idx.push_back(c.next++);
        if (force) want_at.push_back(i);
    }
    if (keys.empty()) {
        (every ? c.hits : c.misses) += n;
        *all = every;
        return 0;
    }
    if (!force) {
        if (build_tables(c, suite, keys, idx, c.build_stream, true) == 0) {
            for (size_t q = 0; q < keys.size(); ++q) c.pending.emplace(keys[q], idx[q]);
            c.build_keys = keys;
            c.build_gen = c.gen;
            c.building = true;
        }
        c.misses += n;
        return 0;
    }
    const int rc = build_tables(c, suite, keys, idx, st, false);
    if (rc) return rc;
    for (size_t q = 0; q < keys.size(); ++q) {
        c.slot_of.emplace(keys[q], idx[q]);
        c.seen.erase(keys[q]);
    }
    c.builds += keys.size();
    c.registered += static_cast<int>(keys.size());
    every = true;
    for (size_t i : want_at) {
        Key64 k;
        std::memcpy(k.data(), pubs + pub_stride * i, 64);
        out[i] = slot_id(c.gen, c.slot_of.at(k));
    }
    for (size_t i = 0; i < n; ++i) every = every && out[i] >= 0;
    (every ? c.hits : c.misses) += n;
    *all = every;
    return 0;
}

int launch_sig_verify_keyed(int suite, const int32_t* d_slots, const uint8_t* d_hash, const uint8_t* d_sig,
                            uint32_t stride, uint64_t n, uint8_t* d_ok, uint8_t* d_addr, hipStream_t st) {
    if (n == 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    KeyCache& c = *cache_of(dev, suite == BCOSGPU_SUITE_SM2 ? 1 : 0);
    const uint32_t* arena;
    uint32_t cap, gen15;
    {
        std::lock_guard<std::mutex> g(c.mu);
        arena = c.arena;
        cap = static_cast<uint32_t>(c.next);  // a batch holds published ids only; pending ones are below next
        gen15 = gen_tag(c.gen);
    }
    if (!arena) return BCOSGPU_E_ARG;  // no key registered on this device
    const dim3 grid(static_cast<unsigned>((n + 3) / 4)), block(64);
    if (suite == BCOSGPU_SUITE_SM2) {
        const uint32_t* tab;
        int bits;
        if (int rc = tables_sm2_26(&tab, &bits)) return rc;
        hipLaunchKernelGGL(sig_verify_keyed_kernel<BCOSGPU_SUITE_SM2>, grid, block, 0, st, arena, cap, gen15, d_slots, d_hash,
                           d_sig, stride, n, tab, bits, d_ok, d_addr);
    } else {
        const uint32_t *k1, *sm2;
        int bits;
        if (int rc = tables(&k1, &sm2, &bits)) return rc;
        hipLaunchKernelGGL(sig_verify_keyed_kernel<BCOSGPU_SUITE_SECP256K1>, grid, block, 0, st, arena, cap, gen15, d_slots,
                           d_hash, d_sig, stride, n, k1, bits, d_ok, d_addr);
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

uint64_t keyed_generation(int suite) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return ~0ull;
    KeyCache& c = *cache_of(dev, suite == BCOSGPU_SUITE_SM2 ? 1 : 0);
    std::lock_guard<std::mutex> g(c.mu);
    return c.gen;
}

int keyed_cache_info(int device, int suite, int64_t out[5]) {
    if (device < 0 || device >= 64) return BCOSGPU_E_ARG;
    KeyCache& c = *cache_of(device, suite == BCOSGPU_SUITE_SM2 ? 1 : 0);
    std::lock_guard<std::mutex> g(c.mu);
    poll_build(c, false);
    out[0] = static_cast<int64_t>(c.slot_of.size());
    out[1] = c.arena ? c.cap : capacity_env();
    out[2] = static_cast<int64_t>(c.hits);
    out[3] = static_cast<int64_t>(c.misses);
    out[4] = static_cast<int64_t>(c.builds);
    return 0;
}

// Drop every cached key of (device, suite) after the device has drained (no launch reads a table then).
int keyed_clear(int device, int suite) {
    if (device < 0 || device >= 64) return BCOSGPU_E_ARG;
    KeyCache& c = *cache_of(device, suite == BCOSGPU_SUITE_SM2 ? 1 : 0);
    std::lock_guard<std::mutex> g(c.mu);
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != device && hipSetDevice(device) != hipSuccess) return BCOSGPU_E_HIP;
    const hipError_t e = hipDeviceSynchronize();
    if (prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) return BCOSGPU_E_HIP;
    c.slot_of.clear();
    c.pending.clear();  // the device drained: a build in flight has completed, and is dropped unpublished
    c.building = false;
    c.build_keys.clear();
    c.next = 0;
    c.seen.clear();
    c.promoted = c.registered = 0;
    ++c.gen;
    return 0;
}

}  // namespace bcosgpu
