// ecc_pair.hip -- small-batch SM2 tx verify: the pair kernels (8 x 32 and fp26 point arithmetic).
#include "ecc_device.h"
#include "ecp26_trio.h"

namespace bcosgpu {

// ------------------------------------------------------------------ SM2 small-batch (pair) tx verify
// Guomi chains verify blocks of C2 size (FastSM2Crypto, FastSM2Crypto.h:33-44).  SM2 has no efficient
// endomorphism, so t*P is ONE chain of 256 doublings and 65 mixed additions.  A 256-thread workgroup
// owns 64 txs:
//   waves 0, 1  build the affine table 1P..8P (wave 0), then run the t*P chain as a PAIR that splits
//               every a = -3 doubling and mixed addition by dependency level and trades field elements
//               through LDS, synchronised by per-wave LDS counters (not workgroup barriers, so the other
//               two waves are never held up):
//                 dbl  (3M + 5S):  a: delta = Z^2, alpha = 3(X - delta)(X + delta), alpha^2
//                                  b: gamma = Y^2, 4 beta = 4 X gamma, 8 gamma^2
//                                  -> a: Y3 = alpha (4 beta - X3) - 8 gamma^2 | b: Z3 = 2 Y Z  (4 of 8 M/S)
//                 madd (7M + 4S):  as tx_verify_coop_kernel's                                   (6 of 11)
//   wave 2      tx hash, e = SM3(Z_A || h), the on-curve check, the address SM3(pub), comb windows
//               0..15 of s*G, then the sum of both comb halves;
//   wave 3      comb windows 16..31 of s*G.
// Waves 2 and 3 finish long before the chain; one final barrier, then wave 0 adds s*G, compares
// projectively and writes the verdict.  Bit-identical to tx_verify_kernel<1, *>.
struct Sm2PairLds {
    uint32_t tab[8][16][64];   // affine 1P..8P (Montgomery): [entry][x0..7, y0..7][lane]
    uint4 ex[2][2][3][2][64];  // [parity][writer role][slot][quad][lane]
    uint32_t g[25][64];        // s*G, Jacobian + inf (wave 2)
    uint32_t gh[25][64];       // comb windows 16..31 (wave 3)
    uint32_t c[8][64];         // (r - e) mod n, plain (wave 2)
    uint32_t addr[5][64];      // right160(SM3(pub)) (wave 2)
    uint32_t ok2[64];          // wave 2's checks: pub on the curve
    uint32_t seq[4];           // pair counters of waves 0, 1; wave 3 done
};

// One pair of waves: each exchange writes the caller's slots of the current parity, publishes its
// sequence number, waits for the partner's, reads the partner's slots and flips parity.  A parity's
// slots are rewritten only after the partner has published the NEXT exchange, i.e. after it has read
// them.
struct PairCtx {
    Sm2PairLds* L;
    int role, lane;
    uint32_t seq;
    int par;
    __device__ __forceinline__ void put(int s, const fe& a) const {
        uint4* p = &L->ex[par][role][s][0][0] + lane;
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void get(int s, fe& a) const {
        const uint4* p = &L->ex[par][role ^ 1][s][0][0] + lane;
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
    __device__ __forceinline__ void sync() {
        ++seq;
        __hip_atomic_store(&L->seq[role], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&L->seq[role ^ 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq) {
        }
    }
    __device__ __forceinline__ void next() { par ^= 1; }
};

// P = 2 P on SM2 (a = -3, dbl-2001-b with Z3 = 2 Y Z), P replicated on both waves of the pair
__device__ __forceinline__ void pair_dbl_am3(Jac& P, PairCtx& c) {
    using F = FieldP2;
    fe alpha, A2, b4, g8, X3, Y3, Z3, t, u;
    if (c.role == 0) {
        fe d;
        F::sqr(d, P.Z);
        F::sub(t, P.X, d);
        F::add(u, P.X, d);
        F::mul(alpha, t, u);
        F::mul3(alpha, alpha);
        F::sqr(A2, alpha);
        c.put(0, alpha);
        c.put(1, A2);
    } else {
        fe g;
        F::sqr(g, P.Y);
        F::mul(b4, P.X, g);
        F::template shl<2>(b4, b4);
        F::sqr(g8, g);
        F::template shl<3>(g8, g8);
        c.put(0, b4);
        c.put(1, g8);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, b4);
        c.get(1, g8);
    } else {
        c.get(0, alpha);
        c.get(1, A2);
    }
    c.next();
    F::template shl<1>(t, b4);
    F::sub(X3, A2, t);  // alpha^2 - 8 beta
    if (c.role == 0) {
        F::sub(t, b4, X3);
        F::mul(Y3, alpha, t);
        F::sub(Y3, Y3, g8);
        c.put(0, Y3);
    } else {
        F::mul(Z3, P.Y, P.Z);
        F::template shl<1>(Z3, Z3);
        c.put(0, Z3);
    }
    c.sync();
    if (c.role == 0) c.get(0, Z3);
    else c.get(0, Y3);
    c.next();
    fe_copy(P.X, X3);
    fe_copy(P.Y, Y3);
    fe_copy(P.Z, Z3);
}

// R = P + Q (madd-2007-bl with the complete-addition special cases of Curve::madd), Q affine
template <class F, class C>
__device__ __forceinline__ void pair_madd(Jac& R, const Jac& P, const Aff& Q, PairCtx& c) {
    fe Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    F::sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        F::mul(u, Q.x, Z1Z1);  // U2
        F::sub(H, u, P.X);
        F::sqr(HH, H);
        F::add(t, P.Z, H);
        F::sqr(Z3, t);
        F::sub(Z3, Z3, Z1Z1);
        F::sub(Z3, Z3, HH);
        c.put(0, H);
        c.put(1, HH);
        c.put(2, Z3);
    } else {
        F::mul(u, Q.y, P.Z);
        F::mul(u, u, Z1Z1);  // S2
        F::sub(rr, u, P.Y);
        F::template shl<1>(rr, rr);
        F::sqr(R2, rr);
        c.put(0, rr);
        c.put(1, R2);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, rr);
        c.get(1, R2);
    } else {
        c.get(0, H);
        c.get(1, HH);
        c.get(2, Z3);
    }
    c.next();
    F::template shl<2>(I, HH);
    if (c.role == 0) {
        F::mul(J, H, I);
        c.put(0, J);
    } else {
        F::mul(V, P.X, I);
        c.put(0, V);
    }
    c.sync();
    if (c.role == 0) c.get(0, V);
    else c.get(0, J);
    c.next();
    F::sub(X3, R2, J);
    F::template shl<1>(t, V);
    F::sub(X3, X3, t);
    if (c.role == 0) {
        F::sub(t, V, X3);
        F::mul(u, rr, t);  // rr (V - X3)
    } else {
        F::mul(u, P.Y, J);
        F::template shl<1>(u, u);  // 2 Y J
    }
    c.put(0, u);
    c.sync();
    c.get(0, t);
    c.next();
    if (c.role == 0) F::sub(Y3, u, t);
    else F::sub(Y3, t, u);
    // special cases, as Curve::madd (computed identically on both waves, no exchanges)
    const bool hz = F::is_zero(H) && !P.inf;
    const bool rz = F::is_zero(rr);
    Jac D;
    if (hz && rz) C::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe_copy(R.X, X3);
    fe_copy(R.Y, Y3);
    fe_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) C::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe_copy(R.X, Q.x);
        fe_copy(R.Y, Q.y);
        F::set_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void pair_add_digit_sm2(Jac& acc, PairCtx& c, int d) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = base[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    fe ny;
    FieldP2::neg(ny, S.y);
    fe_cmov(S.y, ny, d < 0);
    Jac R;
    pair_madd<FieldP2, CurveSM2>(R, acc, S, c);
    CurveSM2::cmov(acc, R, d != 0);
}

// acc = k * G restricted to the 8-bit comb windows [lo, hi)
template <class C>
__device__ __forceinline__ void comb_range8(Jac& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo,
                                            int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    C::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        Aff T;
        load_aff16(T, tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        Jac S;
        C::madd(S, acc, T);
        C::cmov(acc, S, b != 0u);
    }
}

__device__ __forceinline__ void pair_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = P.X.v[k];
        dst[8 + k][lane] = P.Y.v[k];
        dst[16 + k][lane] = P.Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void pair_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        P.X.v[k] = src[k][lane];
        P.Y.v[k] = src[8 + k][lane];
        P.Z.v[k] = src[16 + k][lane];
    }
    P.inf = src[24][lane] != 0u;
}

__global__ __launch_bounds__(256, 1) void tx_verify_sm2_pair_kernel(const uint8_t* __restrict__ pre,
                                                                    const uint64_t* __restrict__ pre_off,
                                                                    const uint8_t* __restrict__ sig,
                                                                    const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                    const uint32_t* __restrict__ tab,
                                                                    uint8_t* __restrict__ txhash,
                                                                    uint8_t* __restrict__ sender,
                                                                    uint8_t* __restrict__ status) {
    __shared__ Sm2PairLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    if (threadIdx.x < 4) L.seq[threadIdx.x] = 0u;
    __syncthreads();
    // signature r || s || pub (SM2Crypto::recover, SignatureDataWithPub.h:55-64); sm2_do_verify checks
    uint64_t sa = 0, sb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
    }
    const bool len_ok = active && sb - sa == 128u;
    fe r, s, px, py;
    uint32_t X[8], Y[8];
    if (len_ok) {
        ByteReader rd(sig + sa, 128);
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(k);
        fe_from_be_words(r, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = rd.word(8 + k);
        fe_from_be_words(s, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            X[k] = bswap32(rd.word(16 + k));
            Y[k] = bswap32(rd.word(24 + k));
        }
    } else {
        fe_zero(r);
        fe_zero(s);
#pragma unroll
        for (int k = 0; k < 8; ++k) X[k] = Y[k] = 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px.v[k] = X[7 - k];
        py.v[k] = Y[7 - k];
    }
    bool ok = len_ok && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    Aff P;
    FieldP2::from_plain(P.x, px);
    FieldP2::from_plain(P.y, py);
    Jac acc;
    if (wave <= 1) {
        PairCtx c{&L, wave, lane, 0u, 0};
        if (wave == 0) {
            Aff A[8];
            sm2_affine_table(A, P);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
            });
        }
        c.sync();  // the table is in LDS
        fe k;
        fe_copy(k, t);
        CurveSM2::set_inf(acc);
        pair_add_digit_sm2(acc, c, static_cast<int>(k.v[7] >> 31));  // digit 64 = bit 255
#pragma unroll 1
        for (int w = 63; w >= 0; --w) {
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            pair_dbl_am3(acc, c);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
            const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            pair_add_digit_sm2(acc, c, d);
        }
    } else if (wave == 2) {
        // tx hash (TarsHashable.h:16-41), e = SM3(Z_A || h) (fast_sm2.cpp:34,203), c = (r - e) mod n
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint64_t pa = pre_off[i], pb = pre_off[i + 1];
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            sm3_msg(rd, len, d);
            store_digest(SM3, txhash + 32 * i, d);
        }
        fe h;
#pragma unroll
        for (int k = 0; k < 8; ++k) h.v[k] = d[7 - k];
        uint32_t eb[8];
        sm2_e(eb, X, Y, h);
        fe e, cc;
#pragma unroll
        for (int k = 0; k < 8; ++k) e.v[k] = eb[7 - k];
        reduce_once(e, ParamN2::M);
        FieldN2::sub(cc, r, e);
        lds_store_fe(L.c, cc, lane);
        fe b;
        fe_set(b, kSM2B);
        L.ok2[lane] = CurveSM2::on_curve(P, b) ? 1u : 0u;
        uint32_t ad[5];
        sm3_address(ad, px, py);
#pragma unroll
        for (int k = 0; k < 5; ++k) L.addr[k][lane] = ad[k];
        Jac G0, G1, G;
        comb_range8<CurveSM2>(G0, s, tab, 0, 16);
        while (__hip_atomic_load(&L.seq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
            __builtin_amdgcn_s_sleep(1);
        }
        pair_load_jac(G1, L.gh, lane);
        CurveSM2::add(G, G0, G1);
        pair_store_jac(L.g, G, lane);
    } else {
        Jac G1;
        comb_range8<CurveSM2>(G1, s, tab, 16, 32);
        pair_store_jac(L.gh, G1, lane);
        __hip_atomic_store(&L.seq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (wave == 0 && active) {
        Jac G, Q;
        pair_load_jac(G, L.g, lane);
        CurveSM2::add(Q, G, acc);
        ok = ok && L.ok2[lane] != 0u && !Q.inf;
        // x1 = X / Z^2 must be congruent to r - e (mod n): x1 = c or c + n (when c + n < p)
        fe cc, c2, cm, z2, rhs;
        lds_load_fe(cc, L.c, lane);
        FieldP2::sqr(z2, Q.Z);
        FieldP2::from_plain(cm, cc);
        FieldP2::mul(rhs, cm, z2);
        bool match = FieldP2::eq(rhs, Q.X);
        const uint32_t carry = fe_add_k(c2, cc, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            FieldP2::from_plain(cm, c2);
            FieldP2::mul(rhs, cm, z2);
            match = match || FieldP2::eq(rhs, Q.X);
        }
        ok = ok && match;
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ok ? L.addr[k][lane] : 0u;
        status[i] = ok ? 0 : 1;
    }
}

// ------------------------------------------------------------------ SM2 pair kernel on fp26
// tx_verify_sm2_pair_kernel with the t*P chain, the comb halves and the final check on fp26 (R' =
// 2^286, ecp26.h); the split of each doubling / mixed addition between the pair is the same, with the
// magnitude plan of CurveSM2x (each wave of the pair normalises the same operands, so both hold
// identical limbs).  Exchanged elements are 5 x uint2 (raw limbs, no canonicalisation).
struct Sm2Pair26Lds {
    uint32_t tab[8][16][64];         // affine 1P..8P in the R' domain, canonical words
    uint2 ex[2][2][3][5][64];        // [parity][writer role][slot][limb pair][lane]
    uint32_t g[25][64];
    uint32_t gh[25][64];
    uint32_t c[8][64];
    uint32_t addr[5][64];
    uint32_t ok2[64];
    uint32_t seq[4];
};

struct Pair26Ctx {
    Sm2Pair26Lds* L;
    int role, lane;
    uint32_t seq;
    int par;
    __device__ __forceinline__ void put(int s, const fp26& a) const {
        uint2* p = &L->ex[par][role][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) p[q * 64] = make_uint2(a.v[2 * q], a.v[2 * q + 1]);
    }
    __device__ __forceinline__ void get(int s, fp26& a) const {
        const uint2* p = &L->ex[par][role ^ 1][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint2 w = p[q * 64];
            a.v[2 * q] = w.x;
            a.v[2 * q + 1] = w.y;
        }
    }
    __device__ __forceinline__ void sync() {
        ++seq;
        __hip_atomic_store(&L->seq[role], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&L->seq[role ^ 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq) {
        }
    }
    __device__ __forceinline__ void next() { par ^= 1; }
};

// as pair_dbl_am3 with CurveSM2x::dbl's magnitudes (X <= 5, Y, Z <= 8 -> (2, 2, 2)):
//   a: alpha = 3 (X - d)(X + d) (3), alpha^2 (1) | b: 4 beta (4), 8 gamma^2 (8)
//   -> both: X3 = alpha^2 - 8 beta (2) -> a: Y3 (2) | b: Z3 = 2 Y Z (2)
__device__ __forceinline__ void pair26_dbl(JacP26& P, Pair26Ctx& c) {
    fp26 alpha, A2, b4, g8, X3, Y3, Z3, t, u;
    if (c.role == 0) {
        fp26 d;
        fp26_sqr(d, P.Z);
        fp26_sub<2>(t, P.X, d);
        fp26_add(u, P.X, d);
        fp26_mul(alpha, t, u);
        fp26_mul_int<3>(alpha, alpha);
        fp26_sqr(A2, alpha);
        c.put(0, alpha);
        c.put(1, A2);
    } else {
        fp26 g;
        fp26_sqr(g, P.Y);
        fp26_mul(b4, P.X, g);
        fp26_mul_int<4>(b4, b4);
        fp26_sqr(g8, g);
        fp26_mul_int<8>(g8, g8);
        c.put(0, b4);
        c.put(1, g8);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, b4);
        c.get(1, g8);
    } else {
        c.get(0, alpha);
        c.get(1, A2);
    }
    c.next();
    F26_SETM(alpha, 3);
    F26_SETM(A2, 1);
    F26_SETM(b4, 4);
    F26_SETM(g8, 8);
    fp26_mul_int<2>(t, b4);
    fp26_sub<9>(X3, A2, t);
    fp26_normalize_weak(X3);
    if (c.role == 0) {
        fp26_sub<3>(t, b4, X3);
        fp26_mul(Y3, alpha, t);
        fp26_sub<9>(Y3, Y3, g8);
        fp26_normalize_weak(Y3);
        c.put(0, Y3);
    } else {
        fp26_mul(Z3, P.Y, P.Z);
        fp26_mul_int<2>(Z3, Z3);
        c.put(0, Z3);
    }
    c.sync();
    if (c.role == 0) c.get(0, Z3);
    else c.get(0, Y3);
    c.next();
    F26_SETM(Y3, 2);
    F26_SETM(Z3, 2);
    fp26_copy(P.X, X3);
    fp26_copy(P.Y, Y3);
    fp26_copy(P.Z, Z3);
}

// as pair_madd with CurveSM2x::madd's arrangement (r = 2 rr, Z3 = 2 Z1 H): P (2, 2, <= 8), Q <= 2
//   a: H (5), HH, Z3 (2) | b: rr (5), R2 = 4 rr^2 (4) -> a: J | b: V -> a: rr (V - X3) | b: Y1 J
__device__ __forceinline__ void pair26_madd(JacP26& R, const JacP26& P, const AffP26& Q, Pair26Ctx& c) {
    fp26 Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    fp26_sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        fp26_mul(u, Q.x, Z1Z1);
        fp26_sub<3>(H, u, P.X);
        fp26_sqr(HH, H);
        fp26_mul(Z3, P.Z, H);
        fp26_mul_int<2>(Z3, Z3);
        c.put(0, H);
        c.put(1, HH);
        c.put(2, Z3);
    } else {
        fp26_mul(u, Q.y, P.Z);
        fp26_mul(u, u, Z1Z1);
        fp26_sub<3>(rr, u, P.Y);
        fp26_sqr(R2, rr);
        fp26_mul_int<4>(R2, R2);
        c.put(0, rr);
        c.put(1, R2);
    }
    c.sync();
    if (c.role == 0) {
        c.get(0, rr);
        c.get(1, R2);
    } else {
        c.get(0, H);
        c.get(1, HH);
        c.get(2, Z3);
    }
    c.next();
    F26_SETM(rr, 5);
    F26_SETM(R2, 4);
    F26_SETM(H, 5);
    F26_SETM(HH, 1);
    F26_SETM(Z3, 2);
    fp26_mul_int<4>(I, HH);
    if (c.role == 0) {
        fp26_mul(J, H, I);
        c.put(0, J);
    } else {
        fp26_mul(V, P.X, I);
        c.put(0, V);
    }
    c.sync();
    if (c.role == 0) c.get(0, V);
    else c.get(0, J);
    c.next();
    F26_SETM(V, 1);
    F26_SETM(J, 1);
    fp26_sub<2>(X3, R2, J);
    fp26_mul_int<2>(t, V);
    fp26_sub<3>(X3, X3, t);
    fp26_normalize_weak(X3);
    if (c.role == 0) {
        fp26_sub<3>(t, V, X3);
        fp26_mul(u, rr, t);
    } else {
        fp26_mul(u, P.Y, J);
    }
    c.put(0, u);
    c.sync();
    c.get(0, t);
    c.next();
    F26_SETM(t, 1);
    if (c.role == 0) fp26_sub<2>(Y3, u, t);
    else fp26_sub<2>(Y3, t, u);
    fp26_mul_int<2>(Y3, Y3);
    fp26_normalize_weak(Y3);
    const bool hz = fp26_is_zero(H) && !P.inf;
    const bool rz = fp26_is_zero(rr);
    JacP26 D;
    if (hz && rz) {  // P == Q (rare); back to the pair chain's magnitudes (2, 2, 2)
        CurveSM2x::dbl(D, P);
        fp26_normalize_weak(D.X);
        fp26_normalize_weak(D.Y);
    }
    const bool pinf = P.inf;
    fp26_copy(R.X, X3);
    fp26_copy(R.Y, Y3);
    fp26_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveSM2x::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fp26_copy(R.X, Q.x);
        fp26_copy(R.Y, Q.y);
        fp26_set(R.Z, p26::ONE_R);
        R.inf = false;
    }
}

__device__ __forceinline__ void pair26_add_digit(JacP26& acc, Pair26Ctx& c, int d) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    AffP26 S;
    {
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x[k] = base[k * 64];
            y[k] = base[(8 + k) * 64];
        }
        fp26_from_words(S.x, x);
        fp26_from_words(S.y, y);
    }
    fp26 ny;
    fp26_neg<2>(ny, S.y);
    fp26_cmov(S.y, ny, d < 0);
    fp26_normalize_weak(S.y);
    JacP26 R;
    pair26_madd(R, acc, S, c);
    CurveSM2x::cmov(acc, R, d != 0);
}

// acc = k * G restricted to the 8-bit comb windows [lo, hi) of the R'-domain table
__device__ __forceinline__ void comb_range_sm2_26(JacP26& acc, const fe& k_plain, const uint32_t* __restrict__ tab,
                                                  int lo, int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    CurveSM2x::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        AffP26 T;
        load_affp26(T, tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        JacP26 S;
        CurveSM2x::madd(S, acc, T);
        CurveSM2x::cmov(acc, S, b != 0u);
    }
}

// acc = k * G restricted to the BITS-bit comb windows [lo, hi) of an R'-domain table (8-bit: kCombEntries
// entries per window; 16-bit: kWideEntries), the next window's entry fetched before the current addition
// (the 16-bit table's gathers come from HBM, not L2)
template <int BITS>
__device__ __forceinline__ void comb_range_sm2_26w(JacP26& acc, const fe& k_plain, const uint32_t* __restrict__ tab,
                                                   int lo, int hi) {
    constexpr uint32_t E = 1u << BITS, MASK = E - 1u;
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr_bits<BITS>(k);
    CurveSM2x::set_inf(acc);
    uint32_t b = k.v[0] & MASK;
    shr_bits<BITS>(k);
    const uint4* e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(lo) * E + b) * 16);
    uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t bi = b;
        AffP26 T;
        {
            const uint32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
            const uint32_t y[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            fp26_from_words(T.x, x);
            fp26_from_words(T.y, y);
        }
        const int in = i + 1 < hi ? i + 1 : i;  // last window: a harmless reload
        b = k.v[0] & MASK;
        shr_bits<BITS>(k);
        e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(in) * E + b) * 16);
        q0 = e[0];
        q1 = e[1];
        q2 = e[2];
        q3 = e[3];
        JacP26 S;
        CurveSM2x::madd(S, acc, T);
        CurveSM2x::cmov(acc, S, bi != 0u);
    }
}
// the comb half of wave 2 (half 0) or 3 (half 1): the 16-bit table's 16 windows split 11 / 5 (wave 3
// builds the affine table first), the 8-bit table's 32 split 16 / 16
__device__ __forceinline__ void comb_half_sm2_26(JacP26& acc, const fe& k, const uint32_t* __restrict__ tab, int bits,
                                                 int half) {
    if (bits == kWideBits) comb_range_sm2_26w<kWideBits>(acc, k, tab, half ? 11 : 0, half ? 16 : 11);
    else comb_range_sm2_26w<8>(acc, k, tab, half ? 16 : 0, half ? 32 : 16);
}

__device__ __forceinline__ void pair26_store_jac(uint32_t (*dst)[64], const JacP26& P, int lane) {
    fe X, Y, Z;
    fp26_to_fe(X, P.X);
    fp26_to_fe(Y, P.Y);
    fp26_to_fe(Z, P.Z);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = X.v[k];
        dst[8 + k][lane] = Y.v[k];
        dst[16 + k][lane] = Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void pair26_load_jac(JacP26& P, const uint32_t (*src)[64], int lane) {
    uint32_t x[8], y[8], z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[k] = src[k][lane];
        y[k] = src[8 + k][lane];
        z[k] = src[16 + k][lane];
    }
    fp26_from_words(P.X, x);
    fp26_from_words(P.Y, y);
    fp26_from_words(P.Z, z);
    P.inf = src[24][lane] != 0u;
}

template <class IO>
__global__ __launch_bounds__(256, 1) void tx_verify_sm2_pair26_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab) {
    __shared__ Sm2Pair26Lds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    if (threadIdx.x < 4) L.seq[threadIdx.x] = 0u;
    __syncthreads();
    fe r, s, px, py;
    uint32_t X[8], Y[8];
    bool len_ok = false;  // the signature (and key) as the I/O policy gives them: r || s || pub, or KeyIO's key
    if constexpr (std::is_same_v<IO, KeyIO>) {
        if (active) len_ok = io.sm2_sig(i, r, s, X, Y);
        else zero_sm2_sig(r, s, X, Y);
    } else {  // (kept in this form: the TxIO / SigIO kernels' register allocation depends on it)
        const uint8_t* sp = nullptr;
        len_ok = active && io.sig_span(i, sp) == 128u;
        if (len_ok) parse_sm2_128(sp, r, s, X, Y);
        else zero_sm2_sig(r, s, X, Y);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px.v[k] = X[7 - k];
        py.v[k] = Y[7 - k];
    }
    bool ok = len_ok && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    AffP26 P;
    fp26_from_plain(P.x, px);
    fp26_from_plain(P.y, py);
    JacP26 acc;
    if (wave <= 1) {
        Pair26Ctx c{&L, wave, lane, 0u, 0};
        if (wave == 0) {
            AffP26 A[8];
            sm2_affine_table26(A, P);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                fe x, y;
                fp26_to_fe(x, A[j].x);
                fp26_to_fe(y, A[j].y);
                lds_store_fe(L.tab[j], x, lane);
                lds_store_fe(L.tab[j] + 8, y, lane);
            });
        }
        c.sync();  // the table is in LDS
        fe k;
        fe_copy(k, t);
        CurveSM2x::set_inf(acc);
        pair26_add_digit(acc, c, static_cast<int>(k.v[7] >> 31));  // digit 64 = bit 255
#pragma unroll 1
        for (int w = 63; w >= 0; --w) {
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            pair26_dbl(acc, c);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
            const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            pair26_add_digit(acc, c, d);
        }
    } else if (wave == 2) {
        fe h;
        fe_zero(h);
        if (active) io.template digest<SM3>(i, h);
        uint32_t eb[8];
        sm2_e(eb, X, Y, h);
        fe e, cc;
#pragma unroll
        for (int k = 0; k < 8; ++k) e.v[k] = eb[7 - k];
        reduce_once(e, ParamN2::M);
        FieldN2::sub(cc, r, e);
        lds_store_fe(L.c, cc, lane);
        L.ok2[lane] = sm2_on_curve26(P) ? 1u : 0u;
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (io.want_addr()) sm3_address(ad, px, py);
#pragma unroll
        for (int k = 0; k < 5; ++k) L.addr[k][lane] = ad[k];
        JacP26 G0, G1, G;
        comb_range_sm2_26(G0, s, tab, 0, 16);
        while (__hip_atomic_load(&L.seq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
            __builtin_amdgcn_s_sleep(1);
        }
        pair26_load_jac(G1, L.gh, lane);
        CurveSM2x::add(G, G0, G1);
        pair26_store_jac(L.g, G, lane);
    } else {
        JacP26 G1;
        comb_range_sm2_26(G1, s, tab, 16, 32);
        pair26_store_jac(L.gh, G1, lane);
        __hip_atomic_store(&L.seq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (wave == 0 && active) {
        JacP26 G, Q;
        pair26_load_jac(G, L.g, lane);
        CurveSM2x::add(Q, G, acc);
        ok = ok && L.ok2[lane] != 0u && !Q.inf;
        fe cc, c2;
        lds_load_fe(cc, L.c, lane);
        fp26 z2, cm, rhs, dlt;
        fp26_sqr(z2, Q.Z);
        fp26_from_plain(cm, cc);
        fp26_mul(rhs, cm, z2);
        fp26_sub<13>(dlt, rhs, Q.X);  // Q.X <= 12 (CurveSM2x::add)
        bool match = fp26_is_zero(dlt);
        const uint32_t carry = fe_add_k(c2, cc, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            fp26_from_plain(cm, c2);
            fp26_mul(rhs, cm, z2);
            fp26_sub<13>(dlt, rhs, Q.X);  // Q.X <= 12 (CurveSM2x::add)
            match = match || fp26_is_zero(dlt);
        }
        ok = ok && match;
        uint32_t ad[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) ad[k] = ok ? L.addr[k][lane] : 0u;
        io.finish(i, ok, ad, nullptr, nullptr);
    }
}
// ------------------------------------------------------------------ SM2 lane-trio kernel (fp26)
// tx_verify_sm2_pair26_kernel with the t*P chain on lane trios (ecp26_trio.h) instead of a wave pair:
// 40 txs per workgroup; waves 0 and 1 both build the affine tables of all 40 txs (identical values, so
// neither waits for the other) and then run the chains of txs 0..19 / 20..39, three lanes per tx;
// waves 2 and 3 hash, derive e and the address and run the two s*G comb halves as in the pair kernel.
// The chain's additions skip the P = +-Q tests (trio_madd_sm2<false>): the accumulator is K P with
// |K| >= 16 before each addition of |d| P, |d| <= 8, and |K| < n, so K = +-d (mod n) cannot occur for
// a P of order n (SM2's cofactor is 1; a P off the curve fails its verdict).  Bit-identical to
// tx_verify_kernel<1, *>.
// Phase stamps of workgroup 0 (s_memtime; tools/sm2bench.hip reads them): always compiled in.  The
// chain loops' register allocation is fragile at ~320 VGPRs, and the product kernel is the one the
// probe measures only if both carry the same stamps (a few scalar-guarded stores per wave).
__device__ uint64_t g_sm2_t[4][8];
#define SM2_T(k) \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_sm2_t[threadIdx.x >> 6][k] = clock64()
// low Booth windows of t P per tx run by waves 2 and 3 (sm2_low_chain)
static constexpr int kSm2TrioSplit = 44;
#ifndef kSm2DblUnroll
#define kSm2DblUnroll 1  // doublings per window unrolled in the chain loops (1 = rolled)
#endif
struct Sm2Trio26Lds {
    uint32_t tab[8][20][64];         // affine 1P..8P in the R' domain as fp26 limbs: [entry][x, y][tx]
    uint32_t jtab[8][50][40];        // Jacobian 1P..8P: [entry][X, Y, Z, Z^2, Z^3][tx]
    uint32_t kt[8][64];              // t = r + s mod n
    uint32_t acc[25][64];            // the chains' results (canonical X, Y, Z, inf)
    uint32_t g[25][64];
    uint32_t gh[25][64];
    uint32_t c[8][64];
    uint32_t addr[5][64];
    uint32_t ok2[64];
    uint32_t kb[8][64];              // t again (waves 2 and 3 write it for their own low-window chains)
    uint32_t bacc[25][64];           // the low-window chains' results (canonical X, Y, Z, inf)
    uint32_t seq[8];
};

__device__ __forceinline__ void trio_add_digit_sm2(TrioPtP& acc, const Sm2Trio26Lds& L, int tl, int d,
                                                   const TrioLane& T) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (20 * 64) + tl;
    AffP26 S;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        S.x.v[q] = base[q * 64];
        S.y.v[q] = base[(10 + q) * 64];
    }
    F26_SETM(S.x, 1);
    F26_SETM(S.y, 1);
    fp26 ny;
    fp26_neg<2>(ny, S.y);
    fp26_cmov(S.y, ny, d < 0);
    fp26_normalize_weak(S.y);
    TrioPtP R;
    trio_madd_sm2<false>(R, acc, S, T);
    trio_cmov_sm2(acc, R, d != 0);
}

// the window's addition on the delta-carrying chain (trio_madd_sm2_d): D = Z^2 on lane 0 in and out
__device__ __forceinline__ void trio_add_digit_sm2_d(TrioPtP& acc, fp26& D, const Sm2Trio26Lds& L, int tl, int d,
                                                     const TrioLane& T) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (20 * 64) + tl;
    AffP26 S;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        S.x.v[q] = base[q * 64];
        S.y.v[q] = base[(10 + q) * 64];
    }
    F26_SETM(S.x, 1);
    F26_SETM(S.y, 1);
    fp26 ny;
    fp26_neg<2>(ny, S.y);
    fp26_cmov(S.y, ny, d < 0);
    fp26_normalize_weak(S.y);
    TrioPtP R;
    fp26 Dn;
    trio_madd_sm2_d(R, Dn, acc, D, S, T);
    trio_cmov_sm2(acc, R, d != 0);
    fp26_cmov(D, Dn, d != 0);
}

// the window's addition before the affine table is ready: the Jacobian entry (trio_add_sm2_jd)
__device__ __forceinline__ void trio_add_digit_sm2_jd(TrioPtP& acc, fp26& D, const Sm2Trio26Lds& L, int tl, int d,
                                                      const TrioLane& T) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.jtab[0][0][0] + m * (50 * 40) + tl;
    JacEntP26 E;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        E.X.v[q] = base[q * 40];
        E.Y.v[q] = base[(10 + q) * 40];
        E.Z.v[q] = base[(20 + q) * 40];
        E.ZZ.v[q] = base[(30 + q) * 40];
        E.ZZZ.v[q] = base[(40 + q) * 40];
    }
    F26_SETM(E.X, 1);
    F26_SETM(E.Y, 1);
    F26_SETM(E.Z, 1);
    F26_SETM(E.ZZ, 1);
    F26_SETM(E.ZZZ, 1);
    fp26 ny;
    fp26_neg<2>(ny, E.Y);
    fp26_cmov(E.Y, ny, d < 0);
    fp26_normalize_weak(E.Y);
    TrioPtP R;
    fp26 Dn;
    trio_add_sm2_jd(R, Dn, acc, D, E, T);
    trio_cmov_sm2(acc, R, d != 0);
    fp26_cmov(D, Dn, d != 0);
}

// entry j of the Jacobian table from a trio's point (X, Z, D on lane 0, Y on lane 1), m 1
__device__ __forceinline__ void trio_store_jent(Sm2Trio26Lds& L, int j, const TrioPtP& P, const fp26& D, int tl,
                                                bool real, const TrioLane& T) {
    fp26 a, b, c;
    fp26_copy(a, P.Xr);
    fp26_copy(b, P.P1);  // lane 0: Z, lane 1: Y
    fp26_copy(c, D);
    fp26_normalize(a);
    fp26_normalize(b);
    fp26_normalize(c);
    if (real && T.r0) {
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            L.jtab[j][q][tl] = a.v[q];
            L.jtab[j][20 + q][tl] = b.v[q];
            L.jtab[j][30 + q][tl] = c.v[q];
        }
    }
    if (real && T.r1) {
#pragma unroll
        for (int q = 0; q < 10; ++q) L.jtab[j][10 + q][tl] = b.v[q];
    }
}

__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The low `split` Booth windows of t P for the 20 txs of chain wave (wave - 2), run on wave 2 / 3 once
// their table, hash and comb work is done (they idled for the rest of the kernel before): t's digits
// split as t = sum_{w >= split} d_w 16^w + sum_{w < split} d_w 16^w, the first sum on waves 0 / 1 (their
// windows 63 .. split, then 4 split doublings), the second here -- the same window loop on t shifted up
// by 4 (64 - split) bits, from infinity, on the affine table.  Its first addition is to infinity; after
// it the accumulator is K P with |K| >= 16 before every addition of |d| P, |d| <= 8, |K| < 2^(4 split + 1)
// < n, so trio_madd_sm2_d's skipped P = +-Q cases cannot occur (as on the high chain).  Stores the sum
// as a Jacobian point at L.bacc[.][tx].
__device__ __forceinline__ void sm2_low_chain(Sm2Trio26Lds& L, int wave, int lane, int split) {
    lds_wave_sync();
    const TrioLane T(lane);
    const int pos = lane & 15, trio_idx = pos / 3;
    const bool real = trio_idx < 5;
    const int tl = (wave - 2) * 20 + (lane >> 4) * 5 + (real ? trio_idx : 4);
    fe k;
#pragma unroll
    for (int q = 0; q < 8; ++q) k.v[q] = L.kb[q][tl];
#pragma unroll 1
    for (int j = 64 - split; j > 0; --j) shl4(k);  // window split - 1 at the top
    TrioPtP acc;
    trio_set_inf_sm2(acc);
    fp26 D;
    fp26_set(D, p26::ONE_R);
    {
        const uint32_t top = k.v[7];
        const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
        const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
        shl4(k);
        trio_add_digit_sm2(acc, L, tl, d, T);  // to infinity: the table point (D = 1) or infinity
    }
#pragma unroll 1
    for (int w = split - 2; w >= 0; --w) {
#pragma unroll kSm2DblUnroll
        for (int q = 0; q < 4; ++q) trio_dbl_sm2_d(acc, D, T);
        const uint32_t top = k.v[7];
        const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
        const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
        shl4(k);
        trio_add_digit_sm2_d(acc, D, L, tl, d, T);
    }
    JacP26 J;
    trio_to_jac_sm2(J, acc, T);
    if (T.r0 && real) pair26_store_jac(L.bacc, J, tl);
}

template <class IO, int SPLIT>
__global__ __launch_bounds__(256, 1) void tx_verify_sm2_trio26_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                                        int affine, const uint32_t* __restrict__ ctab,
                                                                        int cbits) {
    constexpr int split = SPLIT;  // a compile-time bound: the chain loop's code is allocation-sensitive
    constexpr int TPW = 40;
    __shared__ Sm2Trio26Lds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * TPW + lane;
    const bool active = lane < TPW && i < n;
    if (threadIdx.x < 8) L.seq[threadIdx.x] = 0u;
    __syncthreads();
    SM2_T(0);
    fe r, s, px, py;
    uint32_t X[8], Y[8];
    bool len_ok = false;  // the signature (and key) as the I/O policy gives them: r || s || pub, or KeyIO's key
    if constexpr (std::is_same_v<IO, KeyIO>) {
        if (active) len_ok = io.sm2_sig(i, r, s, X, Y);
        else zero_sm2_sig(r, s, X, Y);
    } else {  // (kept in this form: the TxIO / SigIO kernels' register allocation depends on it)
        const uint8_t* sp = nullptr;
        len_ok = active && io.sig_span(i, sp) == 128u;
        if (len_ok) parse_sm2_128(sp, r, s, X, Y);
        else zero_sm2_sig(r, s, X, Y);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px.v[k] = X[7 - k];
        py.v[k] = Y[7 - k];
    }
    bool ok = len_ok && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M);
    fe t;
    FieldN2::add(t, r, s);
    ok = ok && !fe_is_zero_raw(t);
    AffP26 P;
    fp26_from_plain(P.x, px);
    fp26_from_plain(P.y, py);
    // entry 0 of both tables is P itself (one lane per tx; every wave writes the same values)
    {
        fp26 x, y, one;
        fp26_copy(x, P.x);
        fp26_copy(y, P.y);
        fp26_normalize(x);
        fp26_normalize(y);
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            L.tab[0][q][lane] = x.v[q];
            L.tab[0][10 + q][lane] = y.v[q];
        }
        if (wave >= 2 && lane < TPW) {
            fp26_set(one, p26::ONE_R);
            fp26_normalize(one);
#pragma unroll
            for (int q = 0; q < 10; ++q) {
                L.jtab[0][q][lane] = x.v[q];
                L.jtab[0][10 + q][lane] = y.v[q];
                L.jtab[0][20 + q][lane] = one.v[q];
                L.jtab[0][30 + q][lane] = one.v[q];
                L.jtab[0][40 + q][lane] = one.v[q];
            }
        }
    }
    if (wave <= 1) {
#pragma unroll
        for (int q = 0; q < 8; ++q) L.kt[q][lane] = t.v[q];
        lds_wave_sync();  // this wave's own LDS writes before its trio lanes read them
        const TrioLane T(lane);
        const int pos = lane & 15, trio_idx = pos / 3;
        const bool real = trio_idx < 5;
        const int tl = wave * 20 + (lane >> 4) * 5 + (real ? trio_idx : 4);
        SM2_T(1);
        fe k;
#pragma unroll
        for (int q = 0; q < 8; ++q) k.v[q] = L.kt[q][tl];
        TrioPtP acc;
        trio_set_inf_sm2(acc);
        trio_add_digit_sm2(acc, L, tl, static_cast<int>(k.v[7] >> 31), T);  // digit 64 = bit 255 (entry 0)
        fp26 D;  // delta = Z^2 of acc on lane 0 (an affine table point or infinity here)
        fp26_set(D, p26::ONE_R);
        bool aff = false;  // wave-uniform: the affine table (wave 3) is ready
#pragma unroll 1
        for (int w = 63; w >= split; --w) {
            // four doublings, three product levels each (delta carried); rolled: the window's code then
            // fits the instruction cache far better (kSm2DblRoll)
#pragma unroll kSm2DblUnroll
            for (int q = 0; q < 4; ++q) trio_dbl_sm2_d(acc, D, T);
            const uint32_t top = k.v[7];
            const uint32_t W = top >> 28, cb = (top >> 27) & 1u;
            const int d = static_cast<int>(W + cb) - static_cast<int>((W >> 3) << 4);
            shl4(k);
            if (w == 63) {  // this wave's Jacobian table (built by wave 2 + this wave) before the first addition
                while (__hip_atomic_load(&L.seq[wave], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (!aff && affine)
                aff = __builtin_amdgcn_readfirstlane(
                          __hip_atomic_load(&L.seq[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0u;
            if (aff)
                trio_add_digit_sm2_d(acc, D, L, tl, d, T);  // four product levels
            else
                trio_add_digit_sm2_jd(acc, D, L, tl, d, T);  // five
        }
        // the high windows' sum times 2^(4 split): the low windows run on waves 2 and 3
        if constexpr (split > 0) {  // (four doublings per iteration, as in a window: one per iteration
                                    // measured 5.2k cycles each against 4.3k inside the window loop)
#pragma unroll 1
            for (int j = split; j > 0; --j) {
#pragma unroll kSm2DblUnroll
                for (int q = 0; q < 4; ++q) trio_dbl_sm2_d(acc, D, T);
            }
        }
        JacP26 J;
        trio_to_jac_sm2(J, acc, T);
        if (T.r0 && real) pair26_store_jac(L.acc, J, tl);
        SM2_T(2);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) L.kb[q][lane] = t.v[q];  // (both waves write the same values)
        {  // waves 2 and 3: the Jacobian tables of chain waves 0 and 1
            lds_wave_sync();
            const TrioLane T(lane);
            const int pos = lane & 15, trio_idx = pos / 3;
            const bool real = trio_idx < 5;
            const int tl = (wave - 2) * 20 + (lane >> 4) * 5 + (real ? trio_idx : 4);
            // 2P .. 8P of chain wave (wave - 2)'s 20 txs as Jacobian points on the trios (three / four product
            // levels each), then Z^3 of every entry, one product per lane
            {
                AffP26 P0;
#pragma unroll
                for (int q = 0; q < 10; ++q) {
                    P0.x.v[q] = L.tab[0][q][tl];
                    P0.y.v[q] = L.tab[0][10 + q][tl];
                }
                F26_SETM(P0.x, 1);
                F26_SETM(P0.y, 1);
                TrioPtP M1, M2, M3, M;
                fp26 D1, D2, D3, Dm;
                trio_from_aff_sm2(M1, P0, T);
                fp26_set(D1, p26::ONE_R);
                trio_dbl_sm2_d(M1, D1, T);  // 2P
                trio_store_jent(L, 1, M1, D1, tl, real, T);
                trio_madd_sm2_d(M2, D2, M1, D1, P0, T);  // 3P
                trio_store_jent(L, 2, M2, D2, tl, real, T);
                M3 = M1;
                fp26_copy(D3, D1);
                trio_dbl_sm2_d(M3, D3, T);  // 4P
                trio_store_jent(L, 3, M3, D3, tl, real, T);
                trio_madd_sm2_d(M, Dm, M3, D3, P0, T);  // 5P
                trio_store_jent(L, 4, M, Dm, tl, real, T);
                trio_dbl_sm2_d(M2, D2, T);  // 6P
                trio_store_jent(L, 5, M2, D2, tl, real, T);
                trio_madd_sm2_d(M, Dm, M2, D2, P0, T);  // 7P
                trio_store_jent(L, 6, M, Dm, tl, real, T);
                trio_dbl_sm2_d(M3, D3, T);  // 8P
                trio_store_jent(L, 7, M3, D3, tl, real, T);
                lds_wave_sync();
                const int role = T.r0 ? 0 : T.r1 ? 1 : 2;
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int j = 1 + role + 3 * r;
                    const int jj = j <= 7 ? j : 7;
                    fp26 z, zz, zzz;
#pragma unroll
                    for (int q = 0; q < 10; ++q) {
                        z.v[q] = L.jtab[jj][20 + q][tl];
                        zz.v[q] = L.jtab[jj][30 + q][tl];
                    }
                    F26_SETM(z, 1);
                    F26_SETM(zz, 1);
                    fp26_mul(zzz, zz, z);
                    fp26_normalize(zzz);
                    if (real && j <= 7) {
#pragma unroll
                        for (int q = 0; q < 10; ++q) L.jtab[jj][40 + q][tl] = zzz.v[q];
                    }
                }
                lds_wave_sync();
                // these 20 Jacobian tables are complete: chain wave (wave - 2) may add them and wave 3 build
                // their affine forms
                if (lane == 0)
                    __hip_atomic_store(&L.seq[wave - 2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (wave == 2) {
            fe h;
            fe_zero(h);
            if (active) io.template digest<SM3>(i, h);
            uint32_t eb[8];
            sm2_e(eb, X, Y, h);
            fe e, cc;
#pragma unroll
            for (int k = 0; k < 8; ++k) e.v[k] = eb[7 - k];
            reduce_once(e, ParamN2::M);
            FieldN2::sub(cc, r, e);
            lds_store_fe(L.c, cc, lane);
            L.ok2[lane] = sm2_on_curve26(P) ? 1u : 0u;
            uint32_t ad[5] = {0, 0, 0, 0, 0};
            if (io.want_addr()) sm3_address(ad, px, py);
#pragma unroll
            for (int k = 0; k < 5; ++k) L.addr[k][lane] = ad[k];
            JacP26 G0, G1, G;
            SM2_T(1);
            comb_half_sm2_26(G0, s, ctab, cbits, 0);
            SM2_T(2);
            while (__hip_atomic_load(&L.seq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
                __builtin_amdgcn_s_sleep(1);
            }
            pair26_load_jac(G1, L.gh, lane);
            CurveSM2x::add(G, G0, G1);
            pair26_store_jac(L.g, G, lane);
            // (then the low windows of txs 0..19 below: the affine table is complete, wave 3 built it before
            // its comb half, whose result was awaited above)
        } else {
            // the affine table of all 40 txs (one lane per tx) from the Jacobian entries (waves 2 and 3):
            // one inversion of Z1 .. Z7, then x = X / Z^2, y = Y / Z^3; the chains switch to it when ready
            while (__hip_atomic_load(&L.seq[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u ||
                   __hip_atomic_load(&L.seq[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
                __builtin_amdgcn_s_sleep(1);
            }
            {
                const int c = lane < TPW ? lane : TPW - 1;
                fp26 pre[8], inv;
                fp26_set(pre[0], p26::ONE_R);
                Unroll<1, 8>::run([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    fp26 z;
#pragma unroll
                    for (int q = 0; q < 10; ++q) z.v[q] = L.jtab[j][20 + q][c];
                    F26_SETM(z, 1);
                    fp26_mul(pre[j], pre[j - 1], z);
                });
                fp26_inv(inv, pre[7]);  // (Z1 ... Z7)^-1
                Unroll<0, 7>::run([&](auto J) {
                    constexpr int j = 7 - decltype(J)::value;
                    fp26 z, X, Y, zi, zi2, zi3, x, y;
#pragma unroll
                    for (int q = 0; q < 10; ++q) {
                        X.v[q] = L.jtab[j][q][c];
                        Y.v[q] = L.jtab[j][10 + q][c];
                        z.v[q] = L.jtab[j][20 + q][c];
                    }
                    F26_SETM(X, 1);
                    F26_SETM(Y, 1);
                    F26_SETM(z, 1);
                    fp26_mul(zi, inv, pre[j - 1]);  // Z_j^-1
                    fp26_mul(inv, inv, z);          // (Z1 .. Z(j-1))^-1
                    fp26_sqr(zi2, zi);
                    fp26_mul(zi3, zi2, zi);
                    fp26_mul(x, X, zi2);
                    fp26_mul(y, Y, zi3);
                    fp26_normalize(x);
                    fp26_normalize(y);
                    if (lane < TPW) {
#pragma unroll
                        for (int q = 0; q < 10; ++q) {
                            L.tab[j][q][lane] = x.v[q];
                            L.tab[j][10 + q][lane] = y.v[q];
                        }
                    }
                });
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&L.seq[3], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            JacP26 G1;
            SM2_T(1);
            comb_half_sm2_26(G1, s, ctab, cbits, 1);
            SM2_T(2);
            pair26_store_jac(L.gh, G1, lane);
            __hip_atomic_store(&L.seq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (split > 0) {
            // the low windows of txs 0..19 (wave 2) / 20..39 (wave 3), from ONE call site: inlined into each
            // wave's branch the two copies took different register allocations (wave 2's ran 25.6k cycles
            // a window against 22.3k)
            SM2_T(6);
            sm2_low_chain(L, wave, lane, split);
            SM2_T(7);
            if (wave == 3) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(&L.seq[4], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {  // s G + the low sums for all 40 txs
                while (__hip_atomic_load(&L.seq[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
                    __builtin_amdgcn_s_sleep(1);
                }
                lds_wave_sync();
                JacP26 B, S, G;
                pair26_load_jac(S, L.g, lane);
                pair26_load_jac(B, L.bacc, lane);
                CurveSM2x::add(G, S, B);
                pair26_store_jac(L.g, G, lane);
            }
        }
        SM2_T(5);
    }
    __syncthreads();
    SM2_T(3);
    if (wave == 0 && active) {
        JacP26 G, A, Q;
        pair26_load_jac(G, L.g, lane);
        pair26_load_jac(A, L.acc, lane);
        CurveSM2x::add(Q, G, A);
        ok = ok && L.ok2[lane] != 0u && !Q.inf;
        fe cc, c2;
        lds_load_fe(cc, L.c, lane);
        fp26 z2, cm, rhs, dlt;
        fp26_sqr(z2, Q.Z);
        fp26_from_plain(cm, cc);
        fp26_mul(rhs, cm, z2);
        fp26_sub<13>(dlt, rhs, Q.X);  // Q.X <= 12 (CurveSM2x::add)
        bool match = fp26_is_zero(dlt);
        const uint32_t carry = fe_add_k(c2, cc, ParamN2::M);
        if (carry == 0u && fe_lt_k(c2, ParamP2::M)) {
            fp26_from_plain(cm, c2);
            fp26_mul(rhs, cm, z2);
            fp26_sub<13>(dlt, rhs, Q.X);  // Q.X <= 12 (CurveSM2x::add)
            match = match || fp26_is_zero(dlt);
        }
        ok = ok && match;
        uint32_t ad[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) ad[k] = ok ? L.addr[k][lane] : 0u;
        io.finish(i, ok, ad, nullptr, nullptr);
        SM2_T(4);
    }
}

// low Booth windows of t P run by waves 2 and 3 (sm2_low_chain): kSm2TrioSplit balances the two wave
// pairs in the phase probe (profiles/r04_sm2_split_sweep.log); BCOSGPU_SM2_SPLIT=0 (read at each launch,
// as BCOSGPU_SM2_JAC_ONLY) runs all 64 windows on waves 0 and 1, the round-3 schedule (A/B and tests)
static int sm2_trio_split() {
    const char* e = getenv("BCOSGPU_SM2_SPLIT");
    return e ? atoi(e) : kSm2TrioSplit;
}

template <class IO>
int launch_verify_small_sm2(const TxKernelPolicy& pol, const IO& io, uint64_t n, hipStream_t st) {
    if (pol.coop == 3 && pol.f26) return launch_sm2_verify_row(io, n, st);  // ecc_row.hip
    const dim3 grid(static_cast<unsigned>((n + 63) / 64));
    if (pol.f26) {  // fp26 point arithmetic over the R'-domain 8-bit table
        const uint32_t* t26;
        const int rc = tables8_sm2_26(&t26);
        if (rc) return rc;
        if (pol.coop >= 2) {
            // BCOSGPU_SM2_JAC_ONLY=1 (tests): every window adds the Jacobian entry (the affine table unused)
            const char* jo = getenv("BCOSGPU_SM2_JAC_ONLY");
            const int affine = jo && atoi(jo) != 0 ? 0 : 1;
            // s G on the 16-bit comb when the wide R'-domain table exists (half the comb windows on waves
            // 2 and 3, so their low-window chains start earlier)
            const uint32_t* ctab = t26;
            int cbits = 8;
            if (tables_sm2_26(&ctab, &cbits)) {
                ctab = t26;
                cbits = 8;
            }
            const dim3 g(static_cast<unsigned>((n + 39) / 40));
            const int sp = sm2_trio_split();
            if (sp == 0)
                hipLaunchKernelGGL((tx_verify_sm2_trio26_kernel<IO, 0>), g, dim3(256), 0, st, io, n, t26, affine, ctab,
                                   cbits);
            else
                hipLaunchKernelGGL((tx_verify_sm2_trio26_kernel<IO, kSm2TrioSplit>), g, dim3(256), 0, st, io, n, t26,
                                   affine, ctab, cbits);
        }
        else
            hipLaunchKernelGGL(tx_verify_sm2_pair26_kernel<IO>, grid, dim3(256), 0, st, io, n, t26);
    } else if constexpr (std::is_same_v<IO, TxIO>) {
        const uint32_t *k1, *sm2;
        const int rc = tables8(&k1, &sm2);
        if (rc) return rc;
        hipLaunchKernelGGL(tx_verify_sm2_pair_kernel, grid, dim3(256), 0, st, io.pre, io.pre_off, io.sig, io.sig_off, n,
                           sm2, io.txhash, io.sender, io.status);
    } else {
        return BCOSGPU_E_ARG;  // the 8 x 32-bit pair kernel is TxIO only (launch_verify never asks)
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
template int launch_verify_small_sm2<TxIO>(const TxKernelPolicy&, const TxIO&, uint64_t, hipStream_t);
template int launch_verify_small_sm2<SigIO>(const TxKernelPolicy&, const SigIO&, uint64_t, hipStream_t);
template int launch_verify_small_sm2<KeyIO>(const TxKernelPolicy&, const KeyIO&, uint64_t, hipStream_t);

}  // namespace bcosgpu
