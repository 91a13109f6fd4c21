// modinv.h -- modular inversion by Bernstein-Yang "safegcd" divsteps (gfx950, one value per lane).
//
// Replaces Fermat exponentiation (~270-340 modular multiplications) with batches of 30 branch-free
// divsteps on the low 32 bits, each followed by a 2x2 transition-matrix update of the full-width
// (f, g) and (d, e) held as 9 signed 30-bit limbs (v_mad_i64_i32 accumulators).  590 divsteps bound
// any 256-bit input; the loop stops early, wave-uniformly, once g == 0 in every lane of the wave
// (further batches are then exact no-ops).  Values are plain residues in [0, m).
#pragma once
#include "fe.h"

namespace bcosgpu {

struct S30 {
    int32_t v[9];
};

struct ModInfo30 {
    int32_t m[9];    // modulus in signed-30 form
    uint32_t inv30;  // m^-1 mod 2^30
};

__device__ __constant__ static const ModInfo30 kMod30K1P = {
    {1073740847, 1073741819, 1073741823, 1073741823, 1073741823, 1073741823, 1073741823, 1073741823, 65535}, 769313487u};
__device__ __constant__ static const ModInfo30 kMod30N1 = {
    {271991105, 1061780019, 881460155, 733428139, 1073741498, 1073741823, 1073741823, 1073741823, 65535}, 712462017u};
__device__ __constant__ static const ModInfo30 kMod30P2 = {
    {1073741823, 1073741823, 15, 1073741760, 1073741823, 1073741823, 1073741823, 1073725439, 65535}, 1073741823u};
__device__ __constant__ static const ModInfo30 kMod30N2 = {
    {970277155, 250597412, 476074677, 16243400, 1073741682, 1073741823, 1073741823, 1073725439, 65535}, 231405195u};

static constexpr int32_t kM30 = 0x3fffffff;

__device__ __forceinline__ void fe_to_s30(S30& r, const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
        uint32_t x = a.v[w] >> sh;
        if (sh > 2 && w + 1 < 8) x |= a.v[w + 1] << (32 - sh);
        r.v[i] = static_cast<int32_t>(x & kM30);
    }
    r.v[8] = static_cast<int32_t>(a.v[7] >> 16);
}
// limbs normalised to [0, 2^30) with a non-negative top limb
__device__ __forceinline__ void s30_to_fe(fe& r, const S30& a) {
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w, i = bit / 30, sh = bit % 30;
        uint32_t x = static_cast<uint32_t>(a.v[i]) >> sh;
        if (i + 1 < 9) x |= static_cast<uint32_t>(a.v[i + 1]) << (30 - sh);
        if (sh > 28 && i + 2 < 9) x |= static_cast<uint32_t>(a.v[i + 2]) << (60 - sh);
        r.v[w] = x;
    }
}

// 30 divsteps on the low bits of f, g; transition matrix (u, v, q, r) scaled by 2^30:
// u f0 + v g0 = f 2^30, q f0 + r g0 = g 2^30.  zeta = -(delta + 1/2).
__device__ __forceinline__ int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, int32_t t[4]) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
    for (int i = 0; i < 30; ++i) {
        uint32_t c1 = static_cast<uint32_t>(zeta >> 31);  // zeta < 0
        const uint32_t c2 = 0u - (g & 1u);                 // g odd
        const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
        g += x & c2;
        q += y & c2;
        r += z & c2;
        c1 &= c2;
        zeta = (zeta ^ static_cast<int32_t>(c1)) - 1;
        f += g & c1;
        u += q & c1;
        v += r & c1;
        g >>= 1;
        u <<= 1;
        v <<= 1;
    }
    t[0] = static_cast<int32_t>(u);
    t[1] = static_cast<int32_t>(v);
    t[2] = static_cast<int32_t>(q);
    t[3] = static_cast<int32_t>(r);
    return zeta;
}

// 30 divsteps as divsteps_30, in variable time (the var-time loop of libsecp256k1's modinv32, restated):
// a run of zeros at the bottom of g is one shift (count trailing zeros, capped at the steps left by a
// sentinel bit), and up to min(eta + 1, steps left, 8) low bits of g are cancelled at once by adding
// w f, w = -g / f (mod 2^8) with f^-1 by Newton from the 5-bit seed (3 f) ^ 2.  eta = -delta, starting at
// -1 (the delta = 1 variant: at most 724 divsteps for 256-bit inputs, hence 25 batches).  Same matrix
// contract as divsteps_30 (u f0 + v g0 = f 2^30, q f0 + r g0 = g 2^30, |u| + |v|, |q| + |r| <= 2^30), so
// update_fg_30 / update_de_30 apply unchanged.  Lanes run in lockstep: the loop ends when every lane has
// done its 30 steps, a finished lane's iterations being no-ops (limit 0).  Fastest where every lane
// holds the same value (the row kernel's one-signature inversions).
template <int U = 3>
__device__ __forceinline__ int32_t divsteps_30_var(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
    int i = 30;
    // one step of the loop; once a lane has done its 30 divsteps (i == 0) further steps are no-ops
    // (zeros 0, no swap, mask 0), so the exit test (a VALU compare feeding a scalar branch, which stalls
    // a lone wave) runs once per U steps
    auto step = [&]() {
        const int zeros = __builtin_ctz(g | (0xffffffffu << i));
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= zeros;
        i -= zeros;
        const bool live = i != 0;
        const bool sw = live && eta < 0;  // (f, g, u, v, q, r) <- (g, -f, q, r, -u, -v), eta <- -eta
        const uint32_t nf = 0u - f, nu = 0u - u, nv = 0u - v;
        eta = sw ? -eta : eta;
        f = sw ? g : f;
        g = sw ? nf : g;
        u = sw ? q : u;
        q = sw ? nu : q;
        v = sw ? r : v;
        r = sw ? nv : r;
        // limit = min(eta + 1, i) >= 1 on a live lane (eta >= 0 here), 0 on a finished one (i == 0):
        // one v_med3 clamp, the mask of its low bits one v_bfm, capped at 8 bits
        const int lim = (eta + 1) < i ? (eta + 1) : i;
        const uint32_t m = ((1u << (lim < 0 ? 0 : lim)) - 1u) & 255u;
        // f^-1 mod 2^10 by Newton from the 5-bit seed (3 f) ^ 2, and w = -g / f mod 2^8: only low bits
        // matter, so 24-bit multiplies (full rate) suffice
        uint32_t x = ((f << 1) + f) ^ 2u;
        x = (x & 0xffffffu) * ((2u - (f & 0xffffffu) * (x & 0xffffffu)) & 0xffffffu);
        const uint32_t w = ((g & 0xffffffu) * ((0u - x) & 0xffffffu)) & m;
        g += f * w;
        q += u * w;
        r += v * w;
    };
#pragma unroll 1
    for (;;) {
#pragma unroll
        for (int k = 0; k < U; ++k) step();
        // the zeros after the last elimination (a finished lane's i is 0 already)
        const int zeros = __builtin_ctz(g | (0xffffffffu << i));
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= zeros;
        i -= zeros;
        if (__builtin_amdgcn_ballot_w64(i != 0) == 0) break;
    }
    t[0] = static_cast<int32_t>(u);
    t[1] = static_cast<int32_t>(v);
    t[2] = static_cast<int32_t>(q);
    t[3] = static_cast<int32_t>(r);
    return eta;
}

// (f, g) <- t (f, g) / 2^30 (exact)
__device__ __forceinline__ void update_fg_30(S30& f, S30& g, const int32_t t[4]) {
    const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
    int64_t cf = u * f.v[0] + v * g.v[0];
    int64_t cg = q * f.v[0] + r * g.v[0];
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        cf += u * f.v[i] + v * g.v[i];
        cg += q * f.v[i] + r * g.v[i];
        f.v[i - 1] = static_cast<int32_t>(cf) & kM30;
        cf >>= 30;
        g.v[i - 1] = static_cast<int32_t>(cg) & kM30;
        cg >>= 30;
    }
    f.v[8] = static_cast<int32_t>(cf);
    g.v[8] = static_cast<int32_t>(cg);
}

// (d, e) <- (t (d, e) + m (md, me)) / 2^30, md/me chosen so the division is exact; keeps d, e in
// (-2m, m).
__device__ __forceinline__ void update_de_30(S30& d, S30& e, const int32_t t[4], const ModInfo30& mi) {
    const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
    const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
    int32_t md = (u & sd) + (v & se);
    int32_t me = (q & sd) + (r & se);
    int64_t cd = static_cast<int64_t>(u) * d.v[0] + static_cast<int64_t>(v) * e.v[0];
    int64_t ce = static_cast<int64_t>(q) * d.v[0] + static_cast<int64_t>(r) * e.v[0];
    md -= static_cast<int32_t>((mi.inv30 * static_cast<uint32_t>(cd) + static_cast<uint32_t>(md)) & kM30);
    me -= static_cast<int32_t>((mi.inv30 * static_cast<uint32_t>(ce) + static_cast<uint32_t>(me)) & kM30);
    cd += static_cast<int64_t>(mi.m[0]) * md;
    ce += static_cast<int64_t>(mi.m[0]) * me;
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        cd += static_cast<int64_t>(u) * d.v[i] + static_cast<int64_t>(v) * e.v[i];
        ce += static_cast<int64_t>(q) * d.v[i] + static_cast<int64_t>(r) * e.v[i];
        cd += static_cast<int64_t>(mi.m[i]) * md;
        ce += static_cast<int64_t>(mi.m[i]) * me;
        d.v[i - 1] = static_cast<int32_t>(cd) & kM30;
        cd >>= 30;
        e.v[i - 1] = static_cast<int32_t>(ce) & kM30;
        ce >>= 30;
    }
    d.v[8] = static_cast<int32_t>(cd);
    e.v[8] = static_cast<int32_t>(ce);
}

// r in (-2m, m) -> sign * r mod m in [0, m)
__device__ __forceinline__ void normalize_30(S30& r, int32_t sign, const ModInfo30& mi) {
    int32_t ca = r.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] += mi.m[i] & ca;
    const int32_t cn = sign >> 31;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = (r.v[i] ^ cn) - cn;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= kM30;
    }
    ca = r.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] += mi.m[i] & ca;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= kM30;
    }
}

// r = x^-1 mod m (x in [0, m); x = 0 gives 0)
__device__ __forceinline__ void modinv_safegcd(fe& r, const fe& x, const ModInfo30& mi) {
    S30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = mi.m[i];
    }
    e.v[0] = 1;
    fe_to_s30(g, x);
    int32_t zeta = -1;
#pragma unroll 1
    for (int it = 0; it < 20; ++it) {
        int32_t t[4];
        zeta = divsteps_30(zeta, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
        update_de_30(d, e, t, mi);
        update_fg_30(f, g, t);
        int32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= g.v[i];
        if (__builtin_amdgcn_ballot_w64(gz != 0) == 0) break;  // every lane done: the rest are no-ops
    }
    normalize_30(d, f.v[8], mi);
    s30_to_fe(r, d);
}

// r = x^-1 mod m, software-pipelined: the (d, e) update of batch i needs only batch i's matrix, so it
// is issued beside batch i + 1's divstep chain (a serial dependency chain on a lone wave, whose issue
// slots the independent update fills); f, g stay on the critical path as before.  Same result as
// modinv_safegcd; 85.0k -> 74.4k cycles on a lone wave (tools/invbench.hip).  It keeps more values
// live, so it is used where registers are not the constraint (the C2 lane-trio kernel, via
// FieldInv<F>::inv_pipe): in the SM2 trio kernel's table build it measured 5 % slower overall.
__device__ __forceinline__ void modinv_safegcd_pipe(fe& r, const fe& x, const ModInfo30& mi) {
    S30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = mi.m[i];
    }
    e.v[0] = 1;
    fe_to_s30(g, x);
    int32_t t[4];
    int32_t zeta = divsteps_30(-1, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
    update_fg_30(f, g, t);
#pragma unroll 1
    for (int it = 1; it < 20; ++it) {
        int32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= g.v[i];
        if (__builtin_amdgcn_ballot_w64(gz != 0) == 0) break;  // every lane done: the rest are no-ops
        int32_t tp[4] = {t[0], t[1], t[2], t[3]};
        zeta = divsteps_30(zeta, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
        update_de_30(d, e, tp, mi);
        update_fg_30(f, g, t);
    }
    update_de_30(d, e, t, mi);
    normalize_30(d, f.v[8], mi);
    s30_to_fe(r, d);
}

// r = x^-1 mod m with divsteps_30_var, the (d, e) update pipelined as modinv_safegcd_pipe; up to 25
// batches (the delta = 1 bound), ending once g == 0 in every lane.
template <int U = 3>
__device__ __forceinline__ void modinv_safegcd_var(fe& r, const fe& x, const ModInfo30& mi) {
    S30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = mi.m[i];
    }
    e.v[0] = 1;
    fe_to_s30(g, x);
    int32_t t[4];
    int32_t eta = divsteps_30_var<U>(-1, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
    update_fg_30(f, g, t);
#pragma unroll 1
    for (int it = 1; it < 25; ++it) {
        int32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= g.v[i];
        if (__builtin_amdgcn_ballot_w64(gz != 0) == 0) break;
        int32_t tp[4] = {t[0], t[1], t[2], t[3]};
        eta = divsteps_30_var<U>(eta, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
        update_de_30(d, e, tp, mi);
        update_fg_30(f, g, t);
    }
    update_de_30(d, e, t, mi);
    normalize_30(d, f.v[8], mi);
    s30_to_fe(r, d);
}

// modinv_safegcd_var split over two waves of a workgroup, for a value every lane of the producing wave
// holds (the row kernel's Z^-1): the producer runs the divsteps and the (f, g) updates -- the serial
// part -- and posts each batch's matrix to an LDS queue; a second wave applies the (d, e) updates from
// the queue meanwhile (in the one-wave loop they could no longer hide beside the divsteps, whose loop
// ends in a branch), and the producer takes d back at the end.  Same result as modinv_safegcd.
struct InvQueue {
    int32_t t[25][4];
    int32_t d[9];
    uint32_t n, done, ready;  // batches posted, all posted, d written (zero before the producer starts)
};
__device__ __forceinline__ void invq_reset(InvQueue& q) {
    q.n = 0u;
    q.done = 0u;
    q.ready = 0u;
}
// producer: returns f's top limb (its sign gives the result's) for modinv_var_split_finish
__device__ __forceinline__ int32_t modinv_var_split_fg(const fe& x, const ModInfo30& mi, InvQueue& q, int lane) {
    S30 f, g;
#pragma unroll
    for (int i = 0; i < 9; ++i) f.v[i] = mi.m[i];
    fe_to_s30(g, x);
    int32_t eta = -1;
#pragma unroll 1
    for (int it = 0; it < 25; ++it) {
        int32_t t[4];
        eta = divsteps_30_var(eta, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) q.t[it][k] = t[k];
            __hip_atomic_store(&q.n, static_cast<uint32_t>(it + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        update_fg_30(f, g, t);
        int32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= g.v[i];
        if (__builtin_amdgcn_ballot_w64(gz != 0) == 0) break;
    }
    if (lane == 0) __hip_atomic_store(&q.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return f.v[8];
}
// consumer (the other wave): every posted batch's (d, e) update, then d to the queue
__device__ __forceinline__ void modinv_var_split_de(const ModInfo30& mi, InvQueue& q, int lane) {
    S30 d, e;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
    }
    e.v[0] = 1;
#pragma unroll 1
    for (uint32_t b = 0; b < 25u; ++b) {
        uint32_t n;
        for (;;) {
            n = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&q.n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (n > b) break;
            if (__builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&q.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0u) {
                n = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&q.n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (n <= b) break;  // all posted batches applied
        int32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = q.t[b][k];
        update_de_30(d, e, t, mi);
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 9; ++i) q.d[i] = d.v[i];
        __hip_atomic_store(&q.ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
__device__ __forceinline__ void modinv_var_split_finish(fe& r, int32_t fsign, const ModInfo30& mi, InvQueue& q) {
    while (__hip_atomic_load(&q.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(1);
    S30 d;
#pragma unroll
    for (int i = 0; i < 9; ++i) d.v[i] = q.d[i];
    normalize_30(d, fsign, mi);
    s30_to_fe(r, d);
}

// modinv_safegcd split over a wave PAIR for per-lane values (the lane-trio kernel's phase-D Z^-1, one
// value per lane): the producer wave runs the constant-time divsteps and the (f, g) updates and posts
// each batch's matrix, per lane, to a ring of kInvRing slots in LDS; its partner wave, whose lanes hold
// the same values' places, applies the (d, e) updates from the ring meanwhile and returns d.  The
// producer waits only when the ring is full (the consumer's update is the shorter).  Same result as
// modinv_safegcd.  ring: [kInvRing][4][64] words, dq: [9][64] words, ctr: 3 words zeroed beforehand
// (batches posted, batches consumed, d ready; posted | 0x80000000 once the producer is done).
constexpr int kInvRing = 8;
__device__ __forceinline__ int32_t modinv_pair_fg(const fe& x, const ModInfo30& mi, int32_t* ring, uint32_t* ctr,
                                                  int lane) {
    S30 f, g;
#pragma unroll
    for (int i = 0; i < 9; ++i) f.v[i] = mi.m[i];
    fe_to_s30(g, x);
    int32_t zeta = -1;
    uint32_t it = 0;
#pragma unroll 1
    for (; it < 20u; ++it) {
        int32_t t[4];
        zeta = divsteps_30(zeta, static_cast<uint32_t>(f.v[0]), static_cast<uint32_t>(g.v[0]), t);
        if (it >= static_cast<uint32_t>(kInvRing)) {  // the slot's previous batch must be consumed
            while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ctr[1], __ATOMIC_ACQUIRE,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP)) + kInvRing <= it)
                __builtin_amdgcn_s_sleep(1);
        }
        int32_t* slot = ring + (it % kInvRing) * 4 * 64 + lane;
#pragma unroll
        for (int k = 0; k < 4; ++k) slot[k * 64] = t[k];
        if (lane == 0) __hip_atomic_store(&ctr[0], it + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        update_fg_30(f, g, t);
        int32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= g.v[i];
        if (__builtin_amdgcn_ballot_w64(gz != 0) == 0) {
            ++it;
            break;
        }
    }
    if (lane == 0) __hip_atomic_store(&ctr[0], it | 0x80000000u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return f.v[8];
}
__device__ __forceinline__ void modinv_pair_de(const ModInfo30& mi, const int32_t* ring, int32_t* dq, uint32_t* ctr,
                                               int lane) {
    S30 d, e;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
    }
    e.v[0] = 1;
#pragma unroll 1
    for (uint32_t b = 0; b < 20u; ++b) {
        uint32_t n;
        for (;;) {
            n = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&ctr[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if ((n & 0x7fffffffu) > b || (n & 0x80000000u) != 0u) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if ((n & 0x7fffffffu) <= b) break;  // the producer is done and every batch is applied
        const int32_t* slot = ring + (b % kInvRing) * 4 * 64 + lane;
        int32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = slot[k * 64];
        // the slot is free once read: the loads complete before the release store below
        if (lane == 0) __hip_atomic_store(&ctr[1], b + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        update_de_30(d, e, t, mi);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) dq[i * 64 + lane] = d.v[i];
    if (lane == 0) __hip_atomic_store(&ctr[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void modinv_pair_finish(fe& r, int32_t fsign, const ModInfo30& mi, const int32_t* dq,
                                                   uint32_t* ctr, int lane) {
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&ctr[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) ==
           0u)
        __builtin_amdgcn_s_sleep(1);
    S30 d;
#pragma unroll
    for (int i = 0; i < 9; ++i) d.v[i] = dq[i * 64 + lane];
    normalize_30(d, fsign, mi);
    s30_to_fe(r, d);
}

// Field inversion used by the kernels (plain or Montgomery form in, same form out).
// For Montgomery fields: safegcd of a*R gives a^-1 R^-1; multiplying by R^3 (Montgomery) gives a^-1 R.
__device__ __constant__ static const uint32_t kR3P2[8] = {0x00000016u, 0x00000012u, 0xfffffff8u, 0x0000000eu,
                                                       0x0000000cu, 0x0000000au, 0x00000009u, 0x0000001bu};
__device__ __constant__ static const uint32_t kR3N1[8] = {0xe9ff41edu, 0x7bc0cfe0u, 0x44d4322cu, 0x00176484u,
                                                       0xf1d0b2dau, 0xb1b31347u, 0x18ef116du, 0x555d800cu};
__device__ __constant__ static const uint32_t kR3N2[8] = {0x0eaa0b85u, 0x6ff874c7u, 0xaabe8d32u, 0x87d0c315u,
                                                       0x97185afcu, 0x4c4fbbb3u, 0xd574ea14u, 0xc813249cu};

template <class F>
struct FieldInv;
template <>
struct FieldInv<FieldK1> {
    __device__ static __forceinline__ void inv(fe& r, const fe& a) {
        fe t;
        fe_copy(t, a);
        FieldK1::normalize(t);
        modinv_safegcd(r, t, kMod30K1P);
    }
    __device__ static __forceinline__ void inv_pipe(fe& r, const fe& a) {
        fe t;
        fe_copy(t, a);
        FieldK1::normalize(t);
        modinv_safegcd_pipe(r, t, kMod30K1P);
    }
    __device__ static __forceinline__ void inv_var(fe& r, const fe& a) {
        fe t;
        fe_copy(t, a);
        FieldK1::normalize(t);
        modinv_safegcd_var(r, t, kMod30K1P);
    }
};
// PIPE: 0 plain, 1 pipelined, 2 variable time
template <class P, int PIPE = 0>
__device__ __forceinline__ void mont_inv_safegcd(fe& r, const fe& a, const ModInfo30& mi, const uint32_t* r3) {
    fe t, k;
    if constexpr (PIPE == 2) modinv_safegcd_var(t, a, mi);
    else if constexpr (PIPE == 1) modinv_safegcd_pipe(t, a, mi);
    else modinv_safegcd(t, a, mi);
    fe_set(k, r3);
    Mont<P>::mul(r, t, k);
}
template <>
struct FieldInv<FieldP2> {
    __device__ static __forceinline__ void inv(fe& r, const fe& a) { mont_inv_safegcd<ParamP2>(r, a, kMod30P2, kR3P2); }
};
template <>
struct FieldInv<FieldN1> {
    __device__ static __forceinline__ void inv(fe& r, const fe& a) { mont_inv_safegcd<ParamN1>(r, a, kMod30N1, kR3N1); }
    __device__ static __forceinline__ void inv_pipe(fe& r, const fe& a) {
        mont_inv_safegcd<ParamN1, 1>(r, a, kMod30N1, kR3N1);
    }
    __device__ static __forceinline__ void inv_var(fe& r, const fe& a) {
        mont_inv_safegcd<ParamN1, 2>(r, a, kMod30N1, kR3N1);
    }
};
template <>
struct FieldInv<FieldN2> {
    __device__ static __forceinline__ void inv(fe& r, const fe& a) { mont_inv_safegcd<ParamN2>(r, a, kMod30N2, kR3N2); }
};

}  // namespace bcosgpu
