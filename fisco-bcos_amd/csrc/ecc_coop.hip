// ecc_coop.hip -- small-batch secp256k1 tx verify: the 4-wave split kernel, the cooperative-pair kernels
// (8 x 32 and fe26 point arithmetic) and the lane-trio kernel.  Built with the DPP combiner off
// (Makefile; hash_kernels.hip too, for the cooperative Keccak): folding the trio's DPP fetches into
// VOP2 arithmetic gave wrong sums on gfx950 (tools/triobench.hip reproduces it: v_subrev_u32_dpp in
// the mixed addition).
#include "ecc_device.h"
#include "ec26_trio.h"

namespace bcosgpu {

// ------------------------------------------------------------------ split (latency) secp256k1 tx verify
// Small batches are latency-bound: 10k txs fill 157 waves on 1,024 SIMDs, so one recovery per lane
// leaves most of the chip idle.  Here a 256-thread workgroup owns 64 txs and its 4 waves (on the
// CU's 4 SIMDs) run independent parts of every recovery concurrently, exchanging through LDS:
//   phase A  wave 1: tx hash, r^-1 (safegcd), u1 = -e/r, u2 = s/r, GLV split of u2
//            wave 2: y = sqrt(x^3 + 7), table 1R..8R, co-Z rescale -> LDS (affine on E')
//   phase C  wave 0: k1 * R      wave 1: k2 * phi(R)   (32 radix-16 windows each, table in LDS)
//            wave 2: u1 * G (comb)
//   phase D  wave 0: sum on E', map to E, add the G part, affine, Keccak address, store
// Results are bit-identical to tx_verify_kernel<0, *>.
struct SplitLds {
    uint32_t tab[8][16][64];  // [entry][x0..7, y0..7][lane]: conflict-free per-lane gathers
    uint32_t zc[8][64];
    uint32_t u1[8][64];
    uint32_t k1[4][64];
    uint32_t k2[4][64];
    uint32_t flags[64];       // bit0 wave-1 checks ok, bit1 wave-2 checks ok, bit2 neg1, bit3 neg2
    uint32_t pt[3][25][64];   // partial results: X, Y, Z, inf
};

__device__ __forceinline__ void lds_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
    lds_store_fe(dst, P.X, lane);
    lds_store_fe(dst + 8, P.Y, lane);
    lds_store_fe(dst + 16, P.Z, lane);
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void lds_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
    lds_load_fe(P.X, src, lane);
    lds_load_fe(P.Y, src + 8, lane);
    lds_load_fe(P.Z, src + 16, lane);
    P.inf = src[24][lane] != 0u;
}

// acc += (+-d) (phi ? lambda : 1) T[|d| - 1], T gathered per lane from the LDS table (on E')
__device__ __forceinline__ void add_digit_lds(Jac& acc, const SplitLds& L, int lane, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (16 * 64) + lane;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = base[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    if (phi) {
        fe b;
        fe_set(b, kGlvBeta);
        FieldK1::mul(S.x, S.x, b);
    }
    fe ny;
    FieldK1::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    CurveK1::madd(R, acc, S);
    CurveK1::cmov(acc, R, d != 0);
}

__device__ __forceinline__ void glv_half_lds(Jac& acc, fe& k, bool neg, bool phi, const SplitLds& L, int lane) {
    CurveK1::set_inf(acc);
    add_digit_lds(acc, L, lane, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
    for (int i = 31; i >= 0; --i) {
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        CurveK1::dbl(acc, acc);
        add_digit_lds(acc, L, lane, booth_digit128(k), neg, phi);
    }
}

__global__ __launch_bounds__(256, 1) void tx_verify_split_kernel(const uint8_t* __restrict__ pre,
                                                                 const uint64_t* __restrict__ pre_off,
                                                                 const uint8_t* __restrict__ sig,
                                                                 const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                 const uint32_t* __restrict__ tab,
                                                                 uint8_t* __restrict__ txhash,
                                                                 uint8_t* __restrict__ sender,
                                                                 uint8_t* __restrict__ status) {
    __shared__ SplitLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    uint64_t sa = 0, sb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
    }
    const uint32_t slen = (sb - sa) > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(sb - sa);
    // ---------------------------------------------------------------- phase A
    if (wave == 1) {
        if (active) {
            const uint64_t a = pre_off[i], b = pre_off[i + 1];
            const uint32_t len = static_cast<uint32_t>(b - a);
            ByteReader rd(pre + a, len);
            uint32_t d[8];
            keccak256_msg(rd, len, d);
            store_digest(KECCAK256, txhash + 32 * i, d);
            fe e, r, s;
            uint32_t v;
            fe_from_be_words(e, d);
            reduce_once(e, ParamN1::M);
            const bool ok = parse_sig65(sig + sa, slen, r, s, v);
            if (!ok) {
                fe_zero(r);
                r.v[0] = 1;
                fe_zero(s);
            }
            fe rm, rinv, u1, u2, k1, k2;
            FieldN1::from_plain(rm, r);
            FieldInv<FieldN1>::inv(rinv, rm);
            FieldN1::mul(u1, e, rinv);
            FieldN1::neg(u1, u1);
            FieldN1::mul(u2, s, rinv);
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
            lds_store_fe(L.u1, u1, lane);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                L.k1[k][lane] = k1.v[k];
                L.k2[k][lane] = k2.v[k];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
    } else if (wave == 2) {
        if (active) {
            fe r, s;
            uint32_t v;
            bool ok = parse_sig65(sig + sa, slen, r, s, v);
            fe x;
            fe_copy(x, r);
            if (v & 2u) {
                ok = ok && fe_lt_k(r, kK1PminusN);
                fe_add_k(x, r, ParamN1::M);
            }
            fe rhs, y, t, seven;
            FieldK1::sqr(t, x);
            FieldK1::mul(rhs, t, x);
            fe_zero(seven);
            seven.v[0] = 7;
            FieldK1::add(rhs, rhs, seven);
            FieldK1::sqrt_cand(y, rhs);
            FieldK1::sqr(t, y);
            ok = ok && FieldK1::eq(t, rhs);
            FieldK1::normalize(y);
            fe ny;
            FieldK1::neg(ny, y);
            FieldK1::normalize(ny);
            fe_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            Aff R, A[8];
            fe_copy(R.x, x);
            fe_copy(R.y, y);
            fe Zc;
            {
                Jac T[8];
                multiples8<CurveK1>(T, R);
                coz_table_k1(A, Zc, T);
            }
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
            });
            lds_store_fe(L.zc, Zc, lane);
            L.pt[2][24][lane] = ok ? 2u : 0u;  // wave-2 verdict travels in a scratch slot until phase C
        }
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase C
    uint32_t flags = 0;
    if (active) flags = L.flags[lane] | L.pt[2][24][lane];
    __syncthreads();
    if (wave <= 1) {
        if (active) {
            fe k;
            fe_zero(k);
#pragma unroll
            for (int q = 0; q < 4; ++q) k.v[q] = wave == 0 ? L.k1[q][lane] : L.k2[q][lane];
            const bool neg = wave == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
            Jac P;
            glv_half_lds(P, k, neg, wave == 1, L, lane);
            lds_store_jac(L.pt[wave], P, lane);
        }
    } else if (wave == 2) {
        if (active) {
            fe u1;
            lds_load_fe(u1, L.u1, lane);
            Jac PG;
            comb_mul<CurveK1, 8>(PG, u1, tab);
            lds_store_jac(L.pt[2], PG, lane);
        }
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase D
    if (wave == 0 && active) {
        Jac P0, P1, PG, Q, R;
        lds_load_jac(P0, L.pt[0], lane);
        lds_load_jac(P1, L.pt[1], lane);
        lds_load_jac(PG, L.pt[2], lane);
        fe Zc;
        lds_load_fe(Zc, L.zc, lane);
        CurveK1::add(Q, P0, P1);  // on E'
        FieldK1::mul(Q.Z, Q.Z, Zc);  // -> E
        CurveK1::add(R, Q, PG);
        const bool ok = (flags & 3u) == 3u && !R.inf;
        Aff A;
        CurveK1::to_aff(A, R);
        FieldK1::normalize(A.x);
        FieldK1::normalize(A.y);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok) keccak_address(ad, A.x, A.y);
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = ad[k];
        status[i] = ok ? 0 : 1;
    }
}

// ------------------------------------------------------------------ cooperative (latency) secp256k1 tx verify
// A lone wave on a SIMD issues a Comba step only every ~15 cycles and a 64-bit-result op every ~10
// (profiles/r01_mulbench.json), so C2's one-wave-per-SIMD batches are bound by the length of the
// serial point-operation chain, not by the SIMD.  Here the two GLV halves each run on a PAIR of
// waves that split every doubling and mixed addition by dependency level and trade intermediate
// field elements through LDS:
//   dbl  (3M + 4S, depth 2): a: A = X^2, F = (3A)^2, Z3 = 2 Y Z | b: B = Y^2, D = 4 X B, 8 B^2
//                            -> both: X3, Y3 = E (D - X3) - 8C        4 instead of 7, one barrier
//   madd (7M + 4S):          a: Z1Z1, U2, HH, Z3 | b: Z1Z1, S2', S2, rr^2 -> a: J | b: V
//                            -> a: rr (V - X3) | b: Y J        6 instead of 11
// Both waves of a pair hold the whole point after every operation (they compute bit-identical
// values), so the four waves run the same barrier schedule.  Phase A needs no square root before
// the table (the R chain runs on an isomorphic curve, see phase A), so the hash, r^-1, the R table,
// the square root and the comb windows of u1*G run side by side on the four waves, and phase C is
// the two cooperative GLV chains only.  Bit-identical to tx_verify_kernel<0, *>.
#ifdef BCOSGPU_COOP_TIMING  // tools/coopbench.hip: phase timestamps of workgroup 0
__device__ uint64_t g_coop_t[4][8];
__device__ uint64_t g_dbl_t[4][8];
#define DBL_T(k) \
    if (c.probe && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][k] = clock64()
#define COOP_T(k) \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_coop_t[threadIdx.x >> 6][k] = clock64()
#else
#define COOP_T(k) \
    do {          \
    } while (0)
#define DBL_T(k) \
    do {         \
    } while (0)
#endif
struct CoopLds {
    uint32_t tab[8][16][64];          // co-Z table on E': [entry][x0..7, y0..7][lane]
    uint32_t zc[8][64];
    uint32_t k[2][4][64];             // GLV halves
    uint32_t flags[64];               // bit0 scalars ok, bit1 R ok, bit2 neg1, bit3 neg2
    uint4 ex[2][2][6][2][64];         // [chain][writer role][slot][word quad][lane]; madd: 0-2 exchange 0, 3: 1, 4: 2; dbl: 0-2 | 3-5
    uint32_t tabphx[8][8][64];        // beta * x of the table entries (chain 1's phi(R) table)
    uint32_t pt[5][25][64];           // chain results 0/1, G partials 2..4 (X, Y, Z, inf)
    uint32_t xe[8][64];               // e = H(m) mod n (wave 3 -> waves 0, 1)
    uint32_t xrinv[8][64];            // r^-1, Montgomery form (wave 0 -> waves 1, 3)
    uint32_t ys[8][64];               // y of R with v's parity (wave 2 -> phase D)
    uint32_t rflag[64];               // R verdict (wave 2)
    uint32_t post[2];                 // phase-A hand-off flags: 0 r^-1 ready, 1 e ready
};

// One-way hand-offs between waves inside phase A: the producer writes its per-lane values, then
// releases the flag; the consumer acquires it.  Workgroup scope, so these are LDS-only fences.
__device__ __forceinline__ void coop_post(uint32_t* f) {
    __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void coop_wait(uint32_t* f) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(1);
}

struct CoopCtx {
    CoopLds* L;
    int chain, role, lane;
    bool probe;  // BCOSGPU_COOP_TIMING: stamp the doubling phases (workgroup 0, one doubling)
    // An exchange slot is rewritten only after the barrier that follows the partner's read of it,
    // so one slot per (exchange, field element) suffices across consecutive operations.
    // Layout [quad][lane] of uint4: one fe is two conflict-free ds_write_b128 / ds_read_b128.
    __device__ __forceinline__ uint4* slot(int x, int r, int f) const {
        return &L->ex[chain][r][x == 0 ? f : 2 + x][0][0] + lane;
    }
    __device__ __forceinline__ void put(int x, int f, const fe& a) const {
        uint4* p = slot(x, role, f);
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void puts(int s, const fe& a) const {  // raw slot index 0..5
        uint4* p = &L->ex[chain][role][s][0][0] + lane;
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[64] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    }
    __device__ __forceinline__ void gets(int s, fe& a) const {
        const uint4* p = &L->ex[chain][role ^ 1][s][0][0] + lane;
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
    __device__ __forceinline__ void get(int x, int f, fe& a) const {  // the partner's value
        const uint4* p = slot(x, role ^ 1, f);
        const uint4 q0 = p[0], q1 = p[64];
        a.v[0] = q0.x; a.v[1] = q0.y; a.v[2] = q0.z; a.v[3] = q0.w;
        a.v[4] = q1.x; a.v[5] = q1.y; a.v[6] = q1.z; a.v[7] = q1.w;
    }
};

// P = 2 P (a = 0, dbl-2009-l with D = 4 X B), P replicated on both waves of the pair; ONE exchange:
//   a: A = X^2, E = 3A, F = E^2, Z3 = 2 Y Z | b: B = Y^2, D = 4 X B, C = B^2, C8 = 8 C
//   -> both: X3 = F - 2D, Y3 = E (D - X3) - C8
// The shifted passes (shl<k>, mul3) replace ten field additions.  S0 is the exchange buffer: slots
// 0-2 (shared with coop_madd's exchange 0) or 3-5 (3, 4 shared with its exchanges 1, 2).  The four
// doublings of a window use 0, 3, 0, 3, so a slot is rewritten only after the barrier that follows
// the partner's last read of it (the madd rewrites 0-2 before its first barrier, two doublings after
// the last read of buffer 0, and 3/4 only after its first/second barrier).
template <int S0>
__device__ __forceinline__ void coop_dbl(Jac& P, const CoopCtx& c) {
    fe E, F, D, C8, Z3, X3, Y3, t;
    DBL_T(0);
    if (c.role == 0) {
        fe A;
        FieldK1::sqr(A, P.X);
        FieldK1::mul3(E, A);
        FieldK1::sqr(F, E);
        c.puts(S0, E);
        c.puts(S0 + 1, F);
        FieldK1::mul(Z3, P.Y, P.Z);
        FieldK1::template shl<1>(Z3, Z3);
        c.puts(S0 + 2, Z3);
    } else {
        fe B, C;
        FieldK1::sqr(B, P.Y);
        FieldK1::mul(D, P.X, B);
        FieldK1::template shl<2>(D, D);
        c.puts(S0, D);
        FieldK1::sqr(C, B);
        FieldK1::template shl<3>(C8, C);
        c.puts(S0 + 1, C8);
    }
    DBL_T(1);
    __syncthreads();
    DBL_T(2);
    if (c.role == 0) {
        c.gets(S0, D);
        c.gets(S0 + 1, C8);
    } else {
        c.gets(S0, E);
        c.gets(S0 + 1, F);
        c.gets(S0 + 2, Z3);
    }
    FieldK1::template shl<1>(t, D);
    FieldK1::sub(X3, F, t);
    FieldK1::sub(t, D, X3);
    FieldK1::mul(Y3, E, t);
    FieldK1::sub(Y3, Y3, C8);
    DBL_T(3);
    fe_copy(P.X, X3);
    fe_copy(P.Y, Y3);
    fe_copy(P.Z, Z3);
    DBL_T(4);
}

// P = P + Q (madd-2007-bl with the complete-addition special cases of CurveK1::madd), Q affine.
__device__ __forceinline__ void coop_madd(Jac& R, const Jac& P, const Aff& Q, const CoopCtx& c) {
    fe Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    FieldK1::sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        FieldK1::mul(u, Q.x, Z1Z1);       // U2
        FieldK1::sub(H, u, P.X);
        FieldK1::sqr(HH, H);
        FieldK1::add(t, P.Z, H);
        FieldK1::sqr(Z3, t);
        FieldK1::sub(Z3, Z3, Z1Z1);
        FieldK1::sub(Z3, Z3, HH);
        c.put(0, 0, H);
        c.put(0, 1, HH);
        c.put(0, 2, Z3);
    } else {
        FieldK1::mul(u, Q.y, P.Z);
        FieldK1::mul(u, u, Z1Z1);         // S2
        FieldK1::sub(rr, u, P.Y);
        FieldK1::template shl<1>(rr, rr);
        FieldK1::sqr(R2, rr);
        c.put(0, 0, rr);
        c.put(0, 1, R2);
    }
    __syncthreads();
    if (c.role == 0) {
        c.get(0, 0, rr);
        c.get(0, 1, R2);
    } else {
        c.get(0, 0, H);
        c.get(0, 1, HH);
        c.get(0, 2, Z3);
    }
    FieldK1::template shl<2>(I, HH);
    if (c.role == 0) {
        FieldK1::mul(J, H, I);
        c.put(1, 0, J);
    } else {
        FieldK1::mul(V, P.X, I);
        c.put(1, 0, V);
    }
    __syncthreads();
    if (c.role == 0) c.get(1, 0, V);
    else c.get(1, 0, J);
    FieldK1::sub(X3, R2, J);
    FieldK1::template shl<1>(t, V);
    FieldK1::sub(X3, X3, t);
    if (c.role == 0) {
        FieldK1::sub(t, V, X3);
        FieldK1::mul(u, rr, t);           // rr (V - X3)
        c.put(2, 0, u);
    } else {
        FieldK1::mul(u, P.Y, J);
        FieldK1::template shl<1>(u, u);   // 2 Y J
        c.put(2, 0, u);
    }
    __syncthreads();
    if (c.role == 0) {
        c.get(2, 0, t);
        FieldK1::sub(Y3, u, t);
    } else {
        c.get(2, 0, t);
        FieldK1::sub(Y3, t, u);
    }
    // special cases, as CurveK1::madd (computed identically on both waves, no barriers)
    const bool hz = FieldK1::is_zero(H) && !P.inf;
    const bool rz = FieldK1::is_zero(rr);
    Jac D;
    if (hz && rz) CurveK1::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe_copy(R.X, X3);
    fe_copy(R.Y, Y3);
    fe_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveK1::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe_copy(R.X, Q.x);
        fe_copy(R.Y, Q.y);
        FieldK1::set_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void coop_add_digit(Jac& acc, const CoopCtx& c, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    const uint32_t* bx = phi ? &c.L->tabphx[0][0][0] + m * (8 * 64) + c.lane : base;
    Aff S;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        S.x.v[k] = bx[k * 64];
        S.y.v[k] = base[(8 + k) * 64];
    }
    fe ny;
    FieldK1::neg(ny, S.y);
    fe_cmov(S.y, ny, (d < 0) != neg);
    Jac R;
    coop_madd(R, acc, S, c);
    CurveK1::cmov(acc, R, d != 0);
}

// acc = u1 * G restricted to comb windows [lo, hi)
__device__ __forceinline__ void comb_range_k1(Jac& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo, int hi) {
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr8(k);
    CurveK1::set_inf(acc);
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t b = k.v[0] & 255u;
        shr8(k);
        const uint4* e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(i) * kCombEntries + b) * 16);
        const uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
        Aff T;
        T.x.v[0] = q0.x; T.x.v[1] = q0.y; T.x.v[2] = q0.z; T.x.v[3] = q0.w;
        T.x.v[4] = q1.x; T.x.v[5] = q1.y; T.x.v[6] = q1.z; T.x.v[7] = q1.w;
        T.y.v[0] = q2.x; T.y.v[1] = q2.y; T.y.v[2] = q2.z; T.y.v[3] = q2.w;
        T.y.v[4] = q3.x; T.y.v[5] = q3.y; T.y.v[6] = q3.z; T.y.v[7] = q3.w;
        Jac S;
        CurveK1::madd(S, acc, T);
        CurveK1::cmov(acc, S, b != 0u);
    }
}

__device__ __forceinline__ void coop_store_jac(uint32_t (*dst)[64], const Jac& P, int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        dst[k][lane] = P.X.v[k];
        dst[8 + k][lane] = P.Y.v[k];
        dst[16 + k][lane] = P.Z.v[k];
    }
    dst[24][lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void coop_load_jac(Jac& P, const uint32_t (*src)[64], int lane) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        P.X.v[k] = src[k][lane];
        P.Y.v[k] = src[8 + k][lane];
        P.Z.v[k] = src[16 + k][lane];
    }
    P.inf = src[24][lane] != 0u;
}

__global__ __launch_bounds__(256, 1) void tx_verify_coop_kernel(const uint8_t* __restrict__ pre,
                                                                const uint64_t* __restrict__ pre_off,
                                                                const uint8_t* __restrict__ sig,
                                                                const uint64_t* __restrict__ sig_off, uint64_t n,
                                                                const uint32_t* __restrict__ tab,
                                                                uint8_t* __restrict__ txhash,
                                                                uint8_t* __restrict__ sender,
                                                                uint8_t* __restrict__ status) {
    __shared__ CoopLds L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool active = i < n;
    COOP_T(0);
    uint64_t sa = 0, sb = 0, pa = 0, pb = 0;
    if (active) {
        sa = sig_off[i];
        sb = sig_off[i + 1];
        pa = pre_off[i];
        pb = pre_off[i + 1];
    }
    const uint32_t slen = (sb - sa) > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(sb - sa);
    if (threadIdx.x == 0) {
        L.post[0] = 0u;
        L.post[1] = 0u;
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase A
    // R = (x, y) is needed through y only at the very end: the R chain runs on the isomorphic curve
    // E_w: Y^2 = X^3 + 7 w^3 (w = x^3 + 7), where R' = (w x, w^2) needs no square root, and a point
    // (X, Y, Z) of E_w is (X, Y, Z y) on E.  So the square root runs beside the table instead of
    // before it.  Schedule: wave 0 inverts r, wave 3 hashes (they swap r^-1 and e through LDS flags),
    // wave 1 builds the R' table and then the GLV split, wave 2 takes the square root; the comb
    // windows of u1 * G go to waves 0 and 3 and the tail of wave 1.
    fe r, s;
    uint32_t v = 0;
    bool ok = false;
    if (active) ok = parse_sig65(sig + sa, slen, r, s, v);
    else { fe_zero(r); fe_zero(s); }
    if (wave == 1 || wave == 2) {
        fe x, rhs, t, seven;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        FieldK1::sqr(t, x);
        FieldK1::mul(rhs, t, x);
        fe_zero(seven);
        seven.v[0] = 7;
        FieldK1::add(rhs, rhs, seven);  // w
        if (wave == 2) {
            fe y;
            FieldK1::sqrt_cand(y, rhs);
            FieldK1::sqr(t, y);
            okr = okr && FieldK1::eq(t, rhs);
            FieldK1::normalize(y);
            fe ny;
            FieldK1::neg(ny, y);
            FieldK1::normalize(ny);
            fe_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            lds_store_fe(L.ys, y, lane);
            L.rflag[lane] = okr ? 2u : 0u;
            COOP_T(6);
        } else {
            Aff R, A[8];
            FieldK1::mul(R.x, rhs, x);  // w x
            FieldK1::sqr(R.y, rhs);     // w^2
            fe Zc;
            {
                Jac T[8];
                multiples8<CurveK1>(T, R);
                coz_table_k1(A, Zc, T);
            }
            fe beta;
            fe_set(beta, kGlvBeta);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                lds_store_fe(L.tab[j], A[j].x, lane);
                lds_store_fe(L.tab[j] + 8, A[j].y, lane);
                fe bx;
                FieldK1::mul(bx, A[j].x, beta);
                lds_store_fe(L.tabphx[j], bx, lane);
            });
            lds_store_fe(L.zc, Zc, lane);
            COOP_T(6);
        }
    }
    if (!ok) {  // scalars of a rejected signature: any well-defined values (the verdict is already 1)
        fe_zero(r);
        r.v[0] = 1;
        fe_zero(s);
    }
    if (wave == 3) {
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (active) {
            const uint32_t len = static_cast<uint32_t>(pb - pa);
            ByteReader rd(pre + pa, len);
            keccak256_msg(rd, len, d);
            store_digest(KECCAK256, txhash + 32 * i, d);
        }
        fe e;
        fe_from_be_words(e, d);
        reduce_once(e, ParamN1::M);
        lds_store_fe(L.xe, e, lane);
        coop_post(&L.post[1]);
        COOP_T(7);
    } else if (wave == 0) {
        fe rm, rinv;
        FieldN1::from_plain(rm, r);
        FieldInv<FieldN1>::inv(rinv, rm);
        lds_store_fe(L.xrinv, rinv, lane);
        coop_post(&L.post[0]);
        COOP_T(7);
    }
    if (wave != 2) {
        coop_wait(&L.post[0]);
        coop_wait(&L.post[1]);
        fe e, rinv, u1;
        lds_load_fe(e, L.xe, lane);
        lds_load_fe(rinv, L.xrinv, lane);
        FieldN1::mul(u1, e, rinv);
        FieldN1::neg(u1, u1);
        if (wave == 1) {
            fe u2, k1, k2;
            FieldN1::mul(u2, s, rinv);
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L.k[0][q][lane] = k1.v[q];
                L.k[1][q][lane] = k2.v[q];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
        // comb windows of u1 * G: wave 0 [0, kCombW0), wave 3 [kCombW0, kCombW1), wave 1 [kCombW1, 32)
        constexpr int kCombW0 = 12, kCombW1 = 24;
        Jac G;
        const int lo = wave == 0 ? 0 : wave == 3 ? kCombW0 : kCombW1;
        const int hi = wave == 0 ? kCombW0 : wave == 3 ? kCombW1 : 32;
        comb_range_k1(G, u1, tab, lo, hi);
        coop_store_jac(L.pt[wave == 0 ? 2 : wave == 3 ? 3 : 4], G, lane);
    }
    COOP_T(1);
    __syncthreads();
    // ---------------------------------------------------------------- phase C: two cooperative GLV chains
    const uint32_t flags = L.flags[lane] | L.rflag[lane];
    CoopCtx c{&L, wave >> 1, wave & 1, lane, false};
    fe k;
    fe_zero(k);
#pragma unroll
    for (int q = 0; q < 4; ++q) k.v[q] = L.k[c.chain][q][lane];
    const bool neg = c.chain == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
    const bool phi = c.chain == 1;
    Jac acc;
    CurveK1::set_inf(acc);
    coop_add_digit(acc, c, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
    for (int w = 31; w >= 0; --w) {
        coop_dbl<0>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = blockIdx.x == 0 && w == 20;
#endif
        coop_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
        c.probe = false;
#endif
        coop_dbl<0>(acc, c);
        coop_dbl<3>(acc, c);
        coop_add_digit(acc, c, booth_digit128(k), neg, phi);
    }
    COOP_T(2);
    if (c.role == 0) coop_store_jac(L.pt[c.chain], acc, lane);
    __syncthreads();
    // ---------------------------------------------------------------- phase D
    if (wave == 1) {  // G part: partials 0 + 1 + 2
        Jac G0, G1, T, U;
        coop_load_jac(G0, L.pt[2], lane);
        coop_load_jac(G1, L.pt[3], lane);
        CurveK1::add(T, G0, G1);
        coop_load_jac(G0, L.pt[4], lane);
        CurveK1::add(U, T, G0);
        coop_store_jac(L.pt[2], U, lane);
    } else if (wave == 0) {  // R part: co-Z curve -> E_w (Z * Zc) -> E (Z * y)
        Jac P0, P1, Q;
        coop_load_jac(P0, L.pt[0], lane);
        coop_load_jac(P1, L.pt[1], lane);
        fe Zc, y;
        lds_load_fe(Zc, L.zc, lane);
        lds_load_fe(y, L.ys, lane);
        CurveK1::add(Q, P0, P1);
        FieldK1::mul(Zc, Zc, y);
        FieldK1::mul(Q.Z, Q.Z, Zc);
        coop_store_jac(L.pt[0], Q, lane);
    }
    __syncthreads();
    if (wave == 0 && active) {
        Jac Q, G, R;
        coop_load_jac(Q, L.pt[0], lane);
        coop_load_jac(G, L.pt[2], lane);
        CurveK1::add(R, Q, G);
        const bool ok = (flags & 3u) == 3u && !R.inf;
        Aff A;
        COOP_T(4);
        CurveK1::to_aff(A, R);
        COOP_T(5);
        FieldK1::normalize(A.x);
        FieldK1::normalize(A.y);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok) keccak_address(ad, A.x, A.y);
        uint32_t* o = reinterpret_cast<uint32_t*>(sender + 20 * i);
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = ad[q];
        status[i] = ok ? 0 : 1;
    }
    COOP_T(3);
}

// ------------------------------------------------------------------ cooperative kernel on fe26
// tx_verify_coop_kernel with the curve work of phases A and C on the 10 x 26-bit field (fe26.h): the
// same schedule, the same wave roles and the same pair split of every doubling and mixed addition, but
// a lone wave (one per SIMD here) no longer waits on carry chains: its field additions are independent
// limb adds and its multiplies are two interleaved mad chains.  Field elements cross between the two
// waves of a pair as their raw limbs (magnitudes travel with them, as the formulas state); the tables
// and phase results in LDS stay canonical 8-word values, so phase D is tx_verify_coop_kernel's.
// Bit-identical to tx_verify_kernel<0, *>.
struct Coop26Lds {
    uint32_t tab[8][16][64];          // co-Z table on E', canonical words: [entry][x0..7, y0..7][lane]
    uint32_t zc[8][64];
    uint32_t k[2][4][64];             // GLV halves
    uint32_t flags[64];               // bit0 scalars ok, bit1 R ok, bit2 neg1, bit3 neg2
    uint2 ex[2][2][6][5][64];         // [chain][writer role][slot][limb pair][lane]: one fe26 = 5 ds_write_b64
    uint32_t tabphx[8][8][64];        // beta * x of the table entries
    uint32_t pt[5][25][64];           // chain results 0/1, G partials 2..4 (canonical X, Y, Z, inf)
    uint32_t xe[8][64];
    uint32_t xrinv[8][64];
    uint32_t ys[8][64];
    uint32_t rflag[64];
    uint32_t post[3];         // phase-A hand-offs: r^-1, e, G partial 0
};

struct Coop26Ctx {
    Coop26Lds* L;
    int chain, role, lane;
    bool probe;  // BCOSGPU_COOP_TIMING
    __device__ __forceinline__ void puts(int s, const fe26& a) const {
        uint2* p = &L->ex[chain][role][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) p[q * 64] = make_uint2(a.v[2 * q], a.v[2 * q + 1]);
    }
    __device__ __forceinline__ void gets(int s, fe26& a) const {
        const uint2* p = &L->ex[chain][role ^ 1][s][0][0] + lane;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint2 w = p[q * 64];
            a.v[2 * q] = w.x;
            a.v[2 * q + 1] = w.y;
        }
    }
};

// as coop_dbl (slot buffers 0-2 / 3-5 alternate the same way); magnitudes as CurveK1x::dbl:
//   a: A = X^2, E = 3A (3), F = E^2, Z3 = 2 Y Z (2) | b: B = Y^2, D = 4 X B (4), C8 = 8 B^2 (8)
//   -> both: X3 = F - 2D (10), Y3 = E (D - X3) - C8 (10)
template <int S0>
__device__ __forceinline__ void coop26_dbl(Jac26& P, const Coop26Ctx& c) {
    fe26 E, F, D, C8, Z3, X3, Y3, t;
    DBL_T(0);
    if (c.role == 0) {
        fe26 A;
        fe26_sqr(A, P.X);
        fe26_mul_int<3>(E, A);
        fe26_sqr(F, E);
        c.puts(S0, E);
        c.puts(S0 + 1, F);
        fe26_mul(Z3, P.Y, P.Z);
        fe26_mul_int<2>(Z3, Z3);
        c.puts(S0 + 2, Z3);
    } else {
        fe26 B, C;
        fe26_sqr(B, P.Y);
        fe26_mul(D, P.X, B);
        fe26_mul_int<4>(D, D);
        c.puts(S0, D);
        fe26_sqr(C, B);
        fe26_mul_int<8>(C8, C);
        c.puts(S0 + 1, C8);
    }
    DBL_T(1);
    __syncthreads();
    DBL_T(2);
    if (c.role == 0) {
        c.gets(S0, D);
        c.gets(S0 + 1, C8);
    } else {
        c.gets(S0, E);
        c.gets(S0 + 1, F);
        c.gets(S0 + 2, Z3);
    }
    fe26_mul_int<2>(t, D);
    fe26_sub<9>(X3, F, t);
    fe26_sub<11>(t, D, X3);
    fe26_mul(Y3, E, t);
    fe26_sub<9>(Y3, Y3, C8);
    DBL_T(3);
    fe26_copy(P.X, X3);
    fe26_copy(P.Y, Y3);
    fe26_copy(P.Z, Z3);
    DBL_T(4);
}

// as coop_madd, with CurveK1x::madd's arrangement (r = 2 rr, Z3 = 2 Z1 H):
//   both: Z1Z1 | a: U2, H (12), HH, Z3 (2) | b: S2, rr (12), R2 = 4 rr^2 (4)
//   -> a: J = H I | b: V = X1 I        (I = 4 HH)
//   -> a: rr (V - X3) | b: Y1 J        -> Y3 = 2 (a - b) (6);  X3 = R2 - J - 2V (9)
__device__ __forceinline__ void coop26_madd(Jac26& R, const Jac26& P, const Aff26& Q, const Coop26Ctx& c) {
    fe26 Z1Z1, H, HH, Z3, rr, R2, I, J, V, X3, Y3, t, u;
    fe26_sqr(Z1Z1, P.Z);
    if (c.role == 0) {
        fe26_mul(u, Q.x, Z1Z1);
        fe26_sub<11>(H, u, P.X);
        fe26_sqr(HH, H);
        fe26_mul(Z3, P.Z, H);
        fe26_mul_int<2>(Z3, Z3);
        c.puts(0, H);
        c.puts(1, HH);
        c.puts(2, Z3);
    } else {
        fe26_mul(u, Q.y, P.Z);
        fe26_mul(u, u, Z1Z1);
        fe26_sub<11>(rr, u, P.Y);
        fe26_sqr(R2, rr);
        fe26_mul_int<4>(R2, R2);
        c.puts(0, rr);
        c.puts(1, R2);
    }
    __syncthreads();
    if (c.role == 0) {
        c.gets(0, rr);
        c.gets(1, R2);
    } else {
        c.gets(0, H);
        c.gets(1, HH);
        c.gets(2, Z3);
    }
    fe26_mul_int<4>(I, HH);
    if (c.role == 0) {
        fe26_mul(J, H, I);
        c.puts(3, J);
    } else {
        fe26_mul(V, P.X, I);
        c.puts(3, V);
    }
    __syncthreads();
    if (c.role == 0) c.gets(3, V);
    else c.gets(3, J);
    fe26_sub<2>(X3, R2, J);
    fe26_mul_int<2>(t, V);
    fe26_sub<3>(X3, X3, t);
    if (c.role == 0) {
        fe26_sub<10>(t, V, X3);
        fe26_mul(u, rr, t);
        c.puts(4, u);
    } else {
        fe26_mul(u, P.Y, J);
        c.puts(4, u);
    }
    __syncthreads();
    c.gets(4, t);
    if (c.role == 0) fe26_sub<2>(Y3, u, t);
    else fe26_sub<2>(Y3, t, u);
    fe26_mul_int<2>(Y3, Y3);
    const bool hz = fe26_is_zero(H) && !P.inf;
    const bool rz = fe26_is_zero(rr);
    Jac26 D;
    if (hz && rz) CurveK1x::dbl(D, P);  // P == Q (rare)
    const bool pinf = P.inf;
    fe26_copy(R.X, X3);
    fe26_copy(R.Y, Y3);
    fe26_copy(R.Z, Z3);
    R.inf = false;
    if (hz) {
        if (rz) CurveK1x::cmov(R, D, true);
        else R.inf = true;
    }
    if (pinf) {
        fe26_copy(R.X, Q.x);
        fe26_copy(R.Y, Q.y);
        fe26_one(R.Z);
        R.inf = false;
    }
}

__device__ __forceinline__ void coop26_add_digit(Jac26& acc, const Coop26Ctx& c, int d, bool neg, bool phi) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &c.L->tab[0][0][0] + m * (16 * 64) + c.lane;
    const uint32_t* bx = phi ? &c.L->tabphx[0][0][0] + m * (8 * 64) + c.lane : base;
    Aff26 S;
    {
        uint32_t x[8], y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x[k] = bx[k * 64];
            y[k] = base[(8 + k) * 64];
        }
        fe26_from_words(S.x, x);
        fe26_from_words(S.y, y);
    }
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    Jac26 R;
    coop26_madd(R, acc, S, c);
    CurveK1x::cmov(acc, R, d != 0);
}


// acc = u1 * G restricted to the BITS-bit comb windows [lo, hi), the next window's entry fetched (raw
// words) before the current addition, as comb_mul26
template <int BITS>
__device__ __forceinline__ void comb_range26w(Jac26& acc, const fe& k_plain, const uint32_t* __restrict__ tab, int lo,
                                              int hi) {
    constexpr uint32_t E = 1u << BITS, MASK = E - 1u;
    fe k;
    fe_copy(k, k_plain);
    for (int i = 0; i < lo; ++i) shr_bits<BITS>(k);
    CurveK1x::set_inf(acc);
    uint32_t b = k.v[0] & MASK;
    shr_bits<BITS>(k);
    const uint4* e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(lo) * E + b) * 16);
    uint4 q0 = e[0], q1 = e[1], q2 = e[2], q3 = e[3];
#pragma unroll 1
    for (int i = lo; i < hi; ++i) {
        const uint32_t bi = b;
        Aff26 T;
        {
            const uint32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
            const uint32_t y[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            fe26_from_words(T.x, x);
            fe26_from_words(T.y, y);
        }
        const int in = i + 1 < hi ? i + 1 : i;  // last window: a harmless reload
        b = k.v[0] & MASK;
        shr_bits<BITS>(k);
        e = reinterpret_cast<const uint4*>(tab + (static_cast<size_t>(in) * E + b) * 16);
        q0 = e[0];
        q1 = e[1];
        q2 = e[2];
        q3 = e[3];
        Jac26 S;
        CurveK1x::madd(S, acc, T);
        CurveK1x::cmov(acc, S, bi != 0u);
    }
}

// canonical 8-word coordinates into a phase-result slot (the layout coop_load_jac reads)
__device__ __forceinline__ void coop26_store_jac(uint32_t (*dst)[64], const Jac26& P, int lane) {
    fe X, Y, Z;
    fe26_to_fe(X, P.X);
    fe26_to_fe(Y, P.Y);
    fe26_to_fe(Z, P.Z);
    Jac J;
    fe_copy(J.X, X);
    fe_copy(J.Y, Y);
    fe_copy(J.Z, Z);
    J.inf = P.inf;
    coop_store_jac(dst, J, lane);
}
__device__ __forceinline__ void coop26_load_jac(Jac26& P, const uint32_t (*src)[64], int lane) {
    Jac J;
    coop_load_jac(J, src, lane);
    fe26_from_fe(P.X, J.X);
    fe26_from_fe(P.Y, J.Y);
    fe26_from_fe(P.Z, J.Z);
    P.inf = J.inf;
}
__device__ __forceinline__ void lds_load_fe26(fe26& a, const uint32_t (*src)[64], int lane) {
    fe w;
    lds_load_fe(w, src, lane);
    fe26_from_fe(a, w);
}
__device__ __forceinline__ void lds_store_fe26(uint32_t (*dst)[64], const fe26& a, int lane) {
    fe w;
    fe26_to_fe(w, a);
    lds_store_fe(dst, w, lane);
}

// ------------------------------------------------------------------ lane-trio phase C
// The GLV chains of the trio kernel: wave w runs chain w & 1 for txs 20 (w >> 1) .. 20 (w >> 1) + 19
// of the workgroup, one trio (three adjacent lanes, ec26_trio.h) per tx; lane position p of DPP row r
// is trio p / 3 (p = 15 a phantom that mirrors trio 4 and stores nothing).
// The trio kernel's LDS: Coop26Lds without the wave-pair exchange slots, and the co-Z table (and
// beta x) kept as canonical fe26 limbs, so a window's lookup is 20 LDS reads and no conversion.
struct Trio26Lds {
    uint32_t tab[8][20][64];          // [entry][x limbs 0..9, y limbs 0..9][tx]
    uint32_t tabphx[8][10][64];       // beta * x
    uint32_t zc[8][64];
    uint32_t k[2][4][64];
    uint32_t flags[64];
    uint32_t pt[5][25][64];
    uint32_t xe[8][64];
    uint32_t xrinv[8][64];
    uint32_t ys[8][64];
    uint32_t rflag[64];
    uint32_t post[3];
    uint32_t invq[2][4];  // phase D: Z^-1 over wave pairs (0, 1) and (2, 3): posted, consumed, d ready
};
// phase D's Z^-1 ring and d (two wave pairs) live in pt, which is free by then
static_assert(2 * (kInvRing * 4 * 64 + 9 * 64) <= sizeof(Trio26Lds::pt) / 4, "Z^-1 queue exceeds pt");
__device__ __forceinline__ void lds_store_limbs26(uint32_t (*dst)[64], const fe26& a, int lane) {
    fe26 t;
    fe26_copy(t, a);
    fe26_normalize(t);
#pragma unroll
    for (int q = 0; q < 10; ++q) dst[q][lane] = t.v[q];
}

// a TrioPt through LDS (phase D of the trio kernel): [S1 limbs, Xs limbs, Zs limbs, inf][lane], the raw
// limbs (magnitudes travel with the values)
constexpr int kTrioWords = 31;
__device__ __forceinline__ void trio_store(uint32_t* buf, const TrioPt& P, int lane) {
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        buf[q * 64 + lane] = P.S1.v[q];
        buf[(10 + q) * 64 + lane] = P.Xs.v[q];
        buf[(20 + q) * 64 + lane] = P.Zs.v[q];
    }
    buf[30 * 64 + lane] = P.inf ? 1u : 0u;
}
__device__ __forceinline__ void trio_load(TrioPt& P, const uint32_t* buf, int lane) {
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        P.S1.v[q] = buf[q * 64 + lane];
        P.Xs.v[q] = buf[(10 + q) * 64 + lane];
        P.Zs.v[q] = buf[(20 + q) * 64 + lane];
    }
    P.inf = buf[30 * 64 + lane] != 0u;
}
// a Jacobian point held whole by every lane of the trio into trio form
__device__ __forceinline__ void trio_from_jac(TrioPt& P, const Jac26& J, const TrioLane& T) {
    trio::sel(P.S1, T.r0, J.X, J.Y);
    fe26_copy(P.Xs, J.X);
    fe26_copy(P.Zs, J.Z);
    P.inf = J.inf;
}

// A window of a GLV chain: acc <- acc + d * (table point), d a Booth digit in [-8, 8].  The madd runs
// without its P = Q / P = -Q tests (trio_madd<false>): acc is K R for the digits K processed so far
// and the table point is |d| R with |d| <= 8; once K != 0 every window makes |K| >= 16 before its
// addition, so K = +-d (mod n) would need 16 <= |K| <= 8 -- impossible for |K| < 2^130 < n and R of
// order n.  (An R that is not on the curve fails its verdict and its chain's value is discarded.)
// K = 0 is the infinity flag, which the madd handles.
__device__ __forceinline__ void trio_add_digit(TrioPt& acc, const Trio26Lds& L, int tl, int d, bool neg, bool phi,
                                               const TrioLane& T) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (20 * 64) + tl;
    const uint32_t* bx = phi ? &L.tabphx[0][0][0] + m * (10 * 64) + tl : base;
    Aff26 S;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        S.x.v[q] = bx[q * 64];
        S.y.v[q] = base[(10 + q) * 64];
    }
    F26_SETM(S.x, 1);
    F26_SETM(S.y, 1);
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    TrioPt R;
    trio_madd<false>(R, acc, S, T);
    trio_cmov(acc, R, d != 0);
}

// the same window step after trio_dbl_zz: the addition in 4 product levels (trio_madd_zz).  (Reading
// the table entry before the window's doublings, to take the LDS latency off the first level, measured
// no gain: 893k cycles either way.)
__device__ __forceinline__ void trio_add_digit_zz(TrioPt& acc, const Trio26Lds& L, int tl, int d, bool neg, bool phi,
                                                  const fe26& ZZ, const TrioLane& T) {
    const uint32_t m = static_cast<uint32_t>((d < 0 ? -d : d) - 1) & 7u;
    const uint32_t* base = &L.tab[0][0][0] + m * (20 * 64) + tl;
    const uint32_t* bx = phi ? &L.tabphx[0][0][0] + m * (10 * 64) + tl : base;
    Aff26 S;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        S.x.v[q] = bx[q * 64];
        S.y.v[q] = base[(10 + q) * 64];
    }
    F26_SETM(S.x, 1);
    F26_SETM(S.y, 1);
    fe26 ny;
    fe26_neg<2>(ny, S.y);
    fe26_cmov(S.y, ny, (d < 0) != neg);
    TrioPt R;
    trio_madd_zz(R, acc, ZZ, S, T);
    trio_cmov(acc, R, d != 0);
}

// TRIO = false: tx_verify_coop26_kernel (64 txs per workgroup, wave-pair chains); TRIO = true:
// tx_verify_trio26_kernel (40 txs per workgroup, lane-trio chains).  Phases A and D are the same code.
// MODE kRecover: public-key recovery (Q = u1 G + u2 R, R from r and v); MODE kVerify (TRIO only):
// libsecp256k1 ecdsa_verify with a KNOWN key P (sig_verify_trio26_kernel, KeyIO): Q = (e/s) G + (r/s) P,
// accept iff x(Q) = r mod n -- no square root (P is given), s^-1 instead of r^-1, and the projective
// x-check instead of the affine inversion and the address hash.
enum { kRecover = 0, kVerify = 1 };
#ifndef kTrioDblUnroll
#define kTrioDblUnroll 3  // phase C doublings per window unrolled (rolled, 1: 0.385 vs 0.383 ms)
#endif
#ifndef BCOSGPU_TRIO_INV_SPLIT
#define BCOSGPU_TRIO_INV_SPLIT 1  // phase-D Z^-1 over wave pairs (0 = the one-wave pipelined loop, A/B)
#endif
template <bool TRIO, int MODE, class IO>
__device__ __forceinline__ void coop26_body(const IO& io, uint64_t n, const uint32_t* __restrict__ tab, int tab_bits) {
    static_assert(MODE == kRecover || TRIO, "known-key verify runs on the trio kernel only");
    constexpr bool kVer = MODE == kVerify;
    constexpr int TPW = TRIO ? 40 : 64;  // txs per workgroup
    __shared__ std::conditional_t<TRIO, Trio26Lds, Coop26Lds> L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * TPW + lane;
    const bool active = lane < TPW && i < n;
    COOP_T(0);
    if (threadIdx.x == 0) {
        L.post[0] = 0u;
        L.post[1] = 0u;
        L.post[2] = 0u;
        if constexpr (TRIO) {
#pragma unroll
            for (int q = 0; q < 8; ++q) (&L.invq[0][0])[q] = 0u;
        }
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase A (as tx_verify_coop_kernel)
    fe r, s;
    uint32_t v = 0;
    bool ok = false;
    if constexpr (kVer) {
        // verify: wave 1 checks the key and builds ITS table (P is given: no square root); r kept for the
        // final x-check (in the LDS slot recovery uses for y)
        fe kx, ky;
        if (active) {
            io.key_rs(i, r, s, kx, ky);
            ok = fe_lt_k(kx, FieldK1::P) && fe_lt_k(ky, FieldK1::P) && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) &&
                 fe_lt_k(r, ParamN1::M) && fe_lt_k(s, kN1HalfPlus);  // low-S (secp256k1_ecdsa_verify)
        } else {
            fe_zero(r);
            fe_zero(s);
            fe_zero(kx);
            fe_zero(ky);
        }
        if (wave == 0) lds_store_fe(L.ys, r, lane);
        if (wave == 1) {
            Aff26 P;
            fe26_from_fe(P.x, kx);
            fe26_from_fe(P.y, ky);
            fe26 l, rr, t, seven;
            fe26_sqr(l, P.y);
            fe26_sqr(t, P.x);
            fe26_mul(rr, t, P.x);
            fe26_set_small(seven, 7u);
            fe26_add(rr, rr, seven);
            fe26_sub<3>(l, l, rr);
            const bool on = fe26_is_zero(l);  // y^2 = x^3 + 7
            if (!(ok && on)) {  // a valid point for the rejected lanes
                fe26_const(P.x, kK1Gx);
                fe26_const(P.y, kK1Gy);
            }
            L.rflag[lane] = on ? 2u : 0u;
            Aff26 A[8];
            fe26 Zc, beta;
            {
                Jac26 T[8];
                multiples8_26(T, P);
                coz_table26(A, Zc, T);
            }
            fe26_const(beta, kGlvBeta);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                fe26 bx;
                fe26_mul(bx, A[j].x, beta);
                lds_store_limbs26(L.tab[j], A[j].x, lane);
                lds_store_limbs26(L.tab[j] + 10, A[j].y, lane);
                lds_store_limbs26(L.tabphx[j], bx, lane);
            });
            lds_store_fe26(L.zc, Zc, lane);
            COOP_T(6);
        }
    } else {
        if (active) ok = io.rsv(i, r, s, v);
        else { fe_zero(r); fe_zero(s); }
    }
    if (!kVer && (wave == 1 || wave == 2)) {
        fe x;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        fe26 X, rhs, t, seven;
        fe26_from_fe(X, x);
        fe26_sqr(t, X);
        fe26_mul(rhs, t, X);
        fe26_set_small(seven, 7u);
        fe26_add(rhs, rhs, seven);  // w (m 2)
        if (wave == 2) {
            fe26 y, ny;
            fe26_sqrt_cand(y, rhs);
            fe26_sqr(t, y);
            fe26_sub<3>(t, t, rhs);
            okr = okr && fe26_is_zero(t);
            fe26_normalize(y);
            fe26_neg<2>(ny, y);
            fe26_normalize(ny);
            fe26_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            lds_store_fe26(L.ys, y, lane);
            L.rflag[lane] = okr ? 2u : 0u;
            COOP_T(6);
        } else {
            Aff26 R, A[8];
            fe26_mul(R.x, rhs, X);  // w x
            fe26_sqr(R.y, rhs);     // w^2
            fe26 Zc, beta;
            {
                Jac26 T[8];
                multiples8_26(T, R);
                coz_table26(A, Zc, T);
            }
            fe26_const(beta, kGlvBeta);
            Unroll<0, 8>::run([&](auto J) {
                constexpr int j = decltype(J)::value;
                fe26 bx;
                fe26_mul(bx, A[j].x, beta);
                if constexpr (TRIO) {
                    lds_store_limbs26(L.tab[j], A[j].x, lane);
                    lds_store_limbs26(L.tab[j] + 10, A[j].y, lane);
                    lds_store_limbs26(L.tabphx[j], bx, lane);
                } else {
                    lds_store_fe26(L.tab[j], A[j].x, lane);
                    lds_store_fe26(L.tab[j] + 8, A[j].y, lane);
                    lds_store_fe26(L.tabphx[j], bx, lane);
                }
            });
            lds_store_fe26(L.zc, Zc, lane);
            COOP_T(6);
        }
    }
    if (!ok) {  // keep the scalar arithmetic well defined on rejected lanes
        fe_zero(r);
        r.v[0] = 1;
        fe_zero(s);
        if (kVer) s.v[0] = 1;
    }
    if (wave == 3) {
        fe e;
        fe_zero(e);
        if (active) io.template digest<KECCAK256>(i, e);
        reduce_once(e, ParamN1::M);
        lds_store_fe(L.xe, e, lane);
        coop_post(&L.post[1]);
        COOP_T(7);
    } else if (wave == 0) {
        fe rm, rinv;  // verify: w = s^-1 in this slot
        FieldN1::from_plain(rm, kVer ? s : r);
        if constexpr (TRIO) FieldInv<FieldN1>::inv_pipe(rinv, rm);  // (pipelined: this kernel has the registers)
        else FieldInv<FieldN1>::inv(rinv, rm);
        lds_store_fe(L.xrinv, rinv, lane);
        coop_post(&L.post[0]);
        COOP_T(7);
    }
    if (kVer || wave != 2) {
        coop_wait(&L.post[0]);
        coop_wait(&L.post[1]);
        fe e, rinv, u1;
        lds_load_fe(e, L.xe, lane);
        lds_load_fe(rinv, L.xrinv, lane);
        FieldN1::mul(u1, e, rinv);  // recover: u1 = -e / r; verify: u1 = e / s
        if (!kVer) FieldN1::neg(u1, u1);
        if (wave == 1) {
            fe u2, k1, k2;
            FieldN1::mul(u2, kVer ? r : s, rinv);  // recover: s / r; verify: r / s
            bool neg1, neg2;
            glv_split(k1, neg1, k2, neg2, u2);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                L.k[0][q][lane] = k1.v[q];
                L.k[1][q][lane] = k2.v[q];
            }
            L.flags[lane] = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        }
        Jac26 G;
        // recover: wave 2 takes the square root, so the comb windows go to waves 0, 3 and 1; verify: wave 2
        // joins (wave 3 also adds wave 0's partial, wave 1 builds the table first)
        if (tab_bits == kWideBits) {  // 16 windows of the 16-bit comb: 7 / 7 / 2; verify 6 / 4 / 5 / 1
            const int lo = kVer ? (wave == 0 ? 0 : wave == 3 ? 6 : wave == 2 ? 10 : 15) : (wave == 0 ? 0 : wave == 3 ? 7 : 14);
            const int hi = kVer ? (wave == 0 ? 6 : wave == 3 ? 10 : wave == 2 ? 15 : 16) : (wave == 0 ? 7 : wave == 3 ? 14 : 16);
            comb_range26w<kWideBits>(G, u1, tab, lo, hi);
        } else {  // 32 windows of the 8-bit comb: 12 / 12 / 8; verify 11 / 8 / 11 / 2
            const int lo = kVer ? (wave == 0 ? 0 : wave == 3 ? 11 : wave == 2 ? 19 : 30) : (wave == 0 ? 0 : wave == 3 ? 12 : 24);
            const int hi = kVer ? (wave == 0 ? 11 : wave == 3 ? 19 : wave == 2 ? 30 : 32) : (wave == 0 ? 12 : wave == 3 ? 24 : 32);
            comb_range26w<8>(G, u1, tab, lo, hi);
        }
        // G0 + G3 on wave 3 while phase A waits for wave 1's last window (one addition off phase D)
        if (wave == 0) {
            coop26_store_jac(L.pt[2], G, lane);
            coop_post(&L.post[2]);
        } else if (wave == 3) {
            Jac26 G0, S;
            coop_wait(&L.post[2]);
            coop26_load_jac(G0, L.pt[2], lane);
            CurveK1x::add(S, G0, G);
            coop26_store_jac(L.pt[3], S, lane);
        } else if (wave == 1) {
            coop26_store_jac(L.pt[4], G, lane);
        } else {  // verify: wave 2's windows
            coop26_store_jac(L.pt[0], G, lane);
        }
    }
    COOP_T(1);
    __syncthreads();
    // ---------------------------------------------------------------- phase C: two cooperative GLV chains
    if constexpr (TRIO) {
        const TrioLane T(lane);
        const int pos = lane & 15, trio_idx = pos / 3;
        const int chain = wave & 1, tl = (wave >> 1) * 20 + (lane >> 4) * 5 + (trio_idx < 5 ? trio_idx : 4);
        const uint32_t tflags = L.flags[tl] | L.rflag[tl];
        TrioPt acc;
        {
            fe k;
            fe_zero(k);
#pragma unroll
            for (int q = 0; q < 4; ++q) k.v[q] = L.k[chain][q][tl];
            const bool neg = chain == 0 ? (tflags & 4u) != 0 : (tflags & 8u) != 0;
            const bool phi = chain == 1;
            trio_set_inf(acc);
            trio_add_digit(acc, L, tl, static_cast<int>(k.v[3] >> 31), neg, phi, T);  // digit 32 = bit 127
#pragma unroll 1
            for (int w = 31; w >= 0; --w) {
                fe26 zz;
#pragma unroll kTrioDblUnroll
                for (int q = 0; q < 3; ++q) trio_dbl(acc, T);
                trio_dbl_zz(acc, zz, T);  // + Z^2 for the addition
                trio_add_digit_zz(acc, L, tl, booth_digit128(k), neg, phi, zz, T);
            }
        }
        COOP_T(2);
        // ------------------------------------------------------------ phase D on the trios
        // chain 0 (waves 0, 2) takes chain 1's point through LDS and adds it (E_w), maps to E (Z Zc y)
        // and adds the G part, which chain 1 (waves 1, 3) sums meanwhile from phase A's two comb
        // partials; all three additions are trio_add (6 product levels instead of 16 products on one
        // lane).  Then the inversion and the affine map on lane 2 of each trio, the address Keccak on
        // lane PAIRS (KeccakPair) of the chain-0 waves, and the outputs from lane 2.  The buffers reuse
        // the table's LDS once every wave is past phase C.
        uint32_t* const xbuf = &L.tab[0][0][0] + (wave >> 1) * kTrioWords * 64;
        uint32_t* const gbuf = &L.tab[0][0][0] + (2 + (wave >> 1)) * kTrioWords * 64;
        uint32_t* const mbuf = &L.tabphx[0][0][0];  // [40][16] pubkey messages, then [40][8] digests
        const uint64_t ti = static_cast<uint64_t>(blockIdx.x) * TPW + tl;
        const bool real = T.r2 && trio_idx < 5, tactive = ti < n;
        fe26 zcy;
        fe ax, ay;
        bool ok2 = false;
        __syncthreads();  // no wave reads the table any more
        if (chain == 1) {
            trio_store(xbuf, acc, lane);
        } else if constexpr (kVer) {
            lds_load_fe26(zcy, L.zc, tl);  // the co-Z table of P itself: Z Zc
        } else {
            fe26 zc, y;
            lds_load_fe26(zc, L.zc, tl);
            lds_load_fe26(y, L.ys, tl);
            fe26_mul(zcy, zc, y);
        }
        __syncthreads();
        if (chain == 1) {  // G = (G0 + G3) + G1 (+ G2, verify) (phase A's partials)
            Jac26 Ga, Gb;
            TrioPt A, B;
            coop26_load_jac(Ga, L.pt[3], tl);
            coop26_load_jac(Gb, L.pt[4], tl);
            trio_from_jac(A, Ga, T);
            trio_from_jac(B, Gb, T);
            trio_add(A, A, B, T);
            if constexpr (kVer) {
                coop26_load_jac(Gb, L.pt[0], tl);
                trio_from_jac(B, Gb, T);
                trio_add(A, A, B, T);
            }
            trio_store(gbuf, A, lane);
        } else {  // R = (k1 R' + k2 phi(R')) on E_w, then (X, Y, Z Zc y) on E
            TrioPt P1;
            trio_load(P1, xbuf, lane);
            trio_add(acc, acc, P1, T);
            fe26_mul(acc.Zs, acc.Zs, zcy);
        }
        __syncthreads();
        if (chain == 0 && kVer) {
            TrioPt G;
            trio_load(G, gbuf, lane);
            trio_add(acc, acc, G, T);
            // x(Q) = X / Z^2 must be r or r + n (when r + n < p): X == c Z^2, projectively, on lane 2
            fe rr, r2, xw, cw;
            lds_load_fe(rr, L.ys, tl);
            fe26 z2, c, rhs;
            fe26_sqr(z2, acc.Zs);
            fe26_from_fe(c, rr);
            fe26_mul(rhs, c, z2);
            fe26_to_fe(xw, acc.Xs);
            fe26_to_fe(cw, rhs);
            bool match = fe_eq_raw(xw, cw);
            const uint32_t carry = fe_add_k(r2, rr, ParamN1::M);
            const bool second = carry == 0u && fe_lt_k(r2, FieldK1::P);
            fe26_from_fe(c, second ? r2 : rr);
            fe26_mul(rhs, c, z2);
            fe26_to_fe(cw, rhs);
            match = match || (second && fe_eq_raw(xw, cw));
            ok2 = (tflags & 3u) == 3u && !acc.inf && match;
        } else if (chain == 0) {
            TrioPt G;
            trio_load(G, gbuf, lane);
            trio_add(acc, acc, G, T);
            ok2 = (tflags & 3u) == 3u && !acc.inf;
            COOP_T(4);
            fe z, zi;
            fe26_to_fe(z, acc.Zs);
#if BCOSGPU_TRIO_INV_SPLIT
            // Z^-1 over the wave pair: the divsteps and (f, g) here, the (d, e) updates on the chain-1
            // partner (same txs, same lanes), through a ring in the chain points' LDS (free after the
            // barrier above): modinv_pair_*
            FieldK1::normalize(z);
            int32_t* const pq = reinterpret_cast<int32_t*>(&L.pt[0][0][0]);
            int32_t* const ring = pq + (wave >> 1) * (kInvRing * 4 * 64);
            int32_t* const dq = pq + 2 * kInvRing * 4 * 64 + (wave >> 1) * 9 * 64;
            const int32_t fs = modinv_pair_fg(z, kMod30K1P, ring, L.invq[wave >> 1], lane);
            modinv_pair_finish(zi, fs, kMod30K1P, dq, L.invq[wave >> 1], lane);
#else
            FieldInv<FieldK1>::inv_pipe(zi, z);
#endif
            COOP_T(5);
            fe26 zi26, zi2, zi3, X, Y;  // lane 2 holds X (Xs), Y (S1), Z
            fe26_from_fe(zi26, zi);
            fe26_sqr(zi2, zi26);
            fe26_mul(X, acc.Xs, zi2);
            fe26_mul(zi3, zi2, zi26);
            fe26_mul(Y, acc.S1, zi3);
            fe26_to_fe(ax, X);
            fe26_to_fe(ay, Y);
            if (real) {
                uint32_t m[16];
                fe_to_be_words(m, ax);
                fe_to_be_words(m + 8, ay);
#pragma unroll
                for (int q = 0; q < 16; ++q) mbuf[16 * tl + q] = m[q];
            }
        }
#if BCOSGPU_TRIO_INV_SPLIT
        else if (!kVer) {  // chain 1: the (d, e) half of the partner's Z^-1
            const int32_t* const pq = reinterpret_cast<const int32_t*>(&L.pt[0][0][0]);
            modinv_pair_de(kMod30K1P, pq + (wave >> 1) * (kInvRing * 4 * 64),
                           reinterpret_cast<int32_t*>(&L.pt[0][0][0]) + 2 * kInvRing * 4 * 64 + (wave >> 1) * 9 * 64,
                           L.invq[wave >> 1], lane);
        }
#endif
        __syncthreads();
        if (chain == 0 && io.want_addr()) {  // Keccak256(x || y) on lane pairs: tx j = lane / 2 of the wave
            const KeccakPair kp;
            const int j = lane >> 1, t = (wave >> 1) * 20 + (j < 20 ? j : 0);
            uint32_t d[4];
            kp.hash(reinterpret_cast<const uint8_t*>(mbuf + 16 * t), 64u, d);
            if (j < 20) {
#pragma unroll
                for (int q = 0; q < 4; ++q) mbuf[640 + 8 * t + 2 * q + (lane & 1)] = d[q];
            }
        }
        __syncthreads();
        if (chain == 0 && real && tactive) {
            uint32_t ad[5] = {0, 0, 0, 0, 0};
            if (ok2 && io.want_addr()) {
#pragma unroll
                for (int q = 0; q < 5; ++q) ad[q] = mbuf[640 + 8 * tl + 3 + q];  // right160
            }
            io.finish(ti, ok2, ad, &ax, &ay);
        }
        COOP_T(3);
    }
    if constexpr (!TRIO) {
        const uint32_t flags = L.flags[lane] | L.rflag[lane];
        {
            Coop26Ctx c{&L, wave >> 1, wave & 1, lane, false};
            fe k;
            fe_zero(k);
#pragma unroll
            for (int q = 0; q < 4; ++q) k.v[q] = L.k[c.chain][q][lane];
            const bool neg = c.chain == 0 ? (flags & 4u) != 0 : (flags & 8u) != 0;
            const bool phi = c.chain == 1;
            Jac26 acc;
            CurveK1x::set_inf(acc);
            coop26_add_digit(acc, c, static_cast<int>(k.v[3] >> 31), neg, phi);  // digit 32 = bit 127
#pragma unroll 1
            for (int w = 31; w >= 0; --w) {
                coop26_dbl<0>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
                c.probe = blockIdx.x == 0 && w == 20;
#endif
                coop26_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
                c.probe = false;
                if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][5] = clock64();
#endif
                coop26_dbl<0>(acc, c);
                coop26_dbl<3>(acc, c);
#ifdef BCOSGPU_COOP_TIMING
                if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][6] = clock64();
#endif
                coop26_add_digit(acc, c, booth_digit128(k), neg, phi);
#ifdef BCOSGPU_COOP_TIMING
                if (blockIdx.x == 0 && w == 20 && (threadIdx.x & 63) == 0) g_dbl_t[threadIdx.x >> 6][7] = clock64();
#endif
            }
            COOP_T(2);
            if (c.role == 0) coop26_store_jac(L.pt[c.chain], acc, lane);
        }
        __syncthreads();
        // ---------------------------------------------------------------- phase D (on fe26 as well)
        if (wave == 1) {  // G part: (partials 0 + 1, phase A) + 2
            Jac26 G01, G2, U;
            coop26_load_jac(G01, L.pt[3], lane);
            coop26_load_jac(G2, L.pt[4], lane);
            CurveK1x::add(U, G01, G2);
            coop26_store_jac(L.pt[2], U, lane);
        } else if (wave == 0) {  // R part: co-Z curve -> E_w (Z * Zc) -> E (Z * y)
            Jac26 P0, P1, Q;
            coop26_load_jac(P0, L.pt[0], lane);
            coop26_load_jac(P1, L.pt[1], lane);
            fe26 Zc, y;
            lds_load_fe26(Zc, L.zc, lane);
            lds_load_fe26(y, L.ys, lane);
            CurveK1x::add(Q, P0, P1);
            fe26_mul(Zc, Zc, y);
            fe26_mul(Q.Z, Q.Z, Zc);
            coop26_store_jac(L.pt[0], Q, lane);
        }
        __syncthreads();
        if (wave == 0 && active) {
            Jac26 Q, G, R;
            coop26_load_jac(Q, L.pt[0], lane);
            coop26_load_jac(G, L.pt[2], lane);
            CurveK1x::add(R, Q, G);
            const bool ok2 = (flags & 3u) == 3u && !R.inf;
            COOP_T(4);
            fe z, zi, ax, ay;
            fe26_to_fe(z, R.Z);
            FieldInv<FieldK1>::inv(zi, z);
            COOP_T(5);
            fe26 zi26, zi2, zi3, X, Y;
            fe26_from_fe(zi26, zi);
            fe26_sqr(zi2, zi26);
            fe26_mul(X, R.X, zi2);
            fe26_mul(zi3, zi2, zi26);
            fe26_mul(Y, R.Y, zi3);
            fe26_to_fe(ax, X);
            fe26_to_fe(ay, Y);
            uint32_t ad[5] = {0, 0, 0, 0, 0};
            if (ok2 && io.want_addr()) keccak_address(ad, ax, ay);
            io.finish(i, ok2, ad, &ax, &ay);
        }
        COOP_T(3);
    }
}

template <class IO>
__global__ __launch_bounds__(256, 1) void tx_verify_coop26_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab) {
    coop26_body<false, kRecover>(io, n, tab, 8);
}

// The trio kernel: phase C's doublings and mixed additions cost one multiplication of latency per
// dependency level (3 per doubling, 5 per addition) with DPP exchanges inside a wave instead of LDS
// exchanges and barriers between waves, and 40 txs per workgroup spread a 10k batch over 250 CUs
// instead of 157.  Bit-identical to tx_verify_kernel<0, *>.
template <class IO>
__global__ __launch_bounds__(256, 1) void tx_verify_trio26_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                                  int tab_bits) {
    coop26_body<true, kRecover>(io, n, tab, tab_bits);
}

// SignatureCrypto::verify(pub, hash, sig) with a known key on lane trios (KeyIO): the sealer-signature
// checks of PBFT (BlockValidator.cpp:141-182, PBFTCacheProcessor.cpp:795-821 -> Secp256k1Crypto.cpp:51-63)
// verify a block's few signatures per call, so this is the latency path.  Bit-identical verdicts to
// sig_verify_kernel<secp256k1, *> (secp256k1_verify_lane).
__global__ __launch_bounds__(256, 1) void sig_verify_trio26_kernel(KeyIO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                                   int tab_bits) {
    coop26_body<true, kVerify>(io, n, tab, tab_bits);
}

int launch_sig_verify_small_secp(const KeyIO& io, uint64_t n, hipStream_t st) {
    const uint32_t *k1, *sm2;
    int bits = 8;
    const int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL(sig_verify_trio26_kernel, dim3(static_cast<unsigned>((n + 39) / 40)), dim3(256), 0, st, io, n, k1,
                       bits);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}


template <class IO>
int launch_verify_small_secp(const TxKernelPolicy& pol, const IO& io, uint64_t n, hipStream_t st) {
    if (pol.coop == 3 && pol.f26) return launch_recover_row(io, n, st);  // ecc_row.hip
    const uint32_t *k1, *sm2;
    const int rc = tables8(&k1, &sm2);
    if (rc) return rc;
    const dim3 grid(static_cast<unsigned>((n + 63) / 64));
    if (pol.coop == 2 && pol.f26) {
        // u1 G on the 16-bit comb when the wide tables exist (16 windows instead of 32 in phase A)
        const uint32_t *wk1, *wsm2;
        int bits = 8;
        const int rw = tables(&wk1, &wsm2, &bits);
        if (rw) return rw;
        hipLaunchKernelGGL(tx_verify_trio26_kernel<IO>, dim3(static_cast<unsigned>((n + 39) / 40)), dim3(256), 0, st, io,
                           n, wk1, bits);
    } else if (pol.coop && pol.f26) {
        hipLaunchKernelGGL(tx_verify_coop26_kernel<IO>, grid, dim3(256), 0, st, io, n, k1);
    } else if constexpr (std::is_same_v<IO, TxIO>) {
        if (pol.coop)
            hipLaunchKernelGGL(tx_verify_coop_kernel, grid, dim3(256), 0, st, io.pre, io.pre_off, io.sig, io.sig_off, n,
                               k1, io.txhash, io.sender, io.status);
        else
            hipLaunchKernelGGL(tx_verify_split_kernel, grid, dim3(256), 0, st, io.pre, io.pre_off, io.sig, io.sig_off,
                               n, k1, io.txhash, io.sender, io.status);
    } else {
        return BCOSGPU_E_ARG;  // the 8 x 32-bit small-batch kernels are TxIO only (launch_verify never asks)
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
template int launch_verify_small_secp<TxIO>(const TxKernelPolicy&, const TxIO&, uint64_t, hipStream_t);
template int launch_verify_small_secp<SigIO>(const TxKernelPolicy&, const SigIO&, uint64_t, hipStream_t);
template int launch_verify_small_secp<EcrecIO>(const TxKernelPolicy&, const EcrecIO&, uint64_t, hipStream_t);

}  // namespace bcosgpu
