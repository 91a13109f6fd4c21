// ecc_row.hip -- the row kernel: secp256k1 public-key recovery (Secp256k1Crypto.cpp:79-93 via wedpr's
// libsecp256k1 secp256k1_ecdsa_recover semantics) for the smallest batches -- the coalesced single
// recover() calls of tx admission (TxValidator.cpp:27-69 -> Transaction::verify), a block's ecRecover
// calls -- where one signature's serial chain of field products is the whole cost.
//
// One signature per 256-thread workgroup (one wave per SIMD).  The GLV chains run on ROW-spread field
// elements (fe_row.h / ec_row.h: an element over a 16-lane DPP row, ~410 cycles per dependent product
// against 676 / 928 for the one-lane fe26 square / product, tools/rowbench.hip), each wave's four rows
// computing one product level of a point operation together.  The rest is the trio kernel's plan
// (ecc_coop.hip) on one lane per wave:
//   phase A  wave 0: r^-1 (safegcd), then u1 = -e / r, u2 = s / r and the GLV split of u2
//            wave 1: R' = (w x, w^2) on E_w: Y^2 = X^3 + 7 w^3 (w = x^3 + 7: no square root needed),
//                    1R' .. 8R', their co-Z rescale and beta x -> the LDS table
//            wave 2: y = sqrt(w) with v's parity (a point (X, Y, Z) of E_w is (X, Y, Z y) on E)
//            wave 3: e = the digest, then u1 G over the comb table
//   phase C  waves 0 / 1: k1 R' and k2 phi(R') on the rows (33 Booth windows, 3 levels per doubling,
//            3 per addition)
//   phase D  wave 0: the sum, (X, Y, Z Zc y) on E, + u1 G, the affine inversion, the Keccak address.
// Outputs bit-identical to every other recovery kernel (tests/test_gpu_row.py against the oracle).
#include "ecc_device.h"
#include "ec_row.h"

namespace bcosgpu {

namespace {

struct RowLds {
    uint32_t tab[8][3][16];  // co-Z table of R' on E_w: x, y, beta x as canonical fe26 limbs (10..15 zero)
    uint32_t res[2][3][16];  // the chains' points (row limbs), phase C -> D
    uint32_t k[2][4];        // GLV halves of u2
    uint32_t u1[8], e[8], zc[8], ys[8];
    uint32_t g[3][8];        // u1 G (canonical words)
    uint32_t kflags;         // wave 0: bit 0 scalars ok, bit 2 neg1, bit 3 neg2
    uint32_t rflag;          // wave 2: R on the curve (bit 1)
    uint32_t ginf, cinf[2];  // u1 G / chain results at infinity
    uint32_t post[3];        // 0: e, 1: k / u1, 2: table
};

__device__ __forceinline__ void row_post(uint32_t* f) {
    __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void row_wait(uint32_t* f) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void put8(uint32_t* d, const fe& a, int lane) {
    if (lane < 8) d[lane] = a.v[lane];
}
__device__ __forceinline__ void get8(fe& a, const uint32_t* d) {
#pragma unroll
    for (int q = 0; q < 8; ++q) a.v[q] = d[q];
}
// a fe26 as canonical limbs into a 16-word row slot
__device__ __forceinline__ void put_limbs(uint32_t* d, const fe26& a, int lane) {
    fe26 t;
    fe26_copy(t, a);
    fe26_normalize(t);
    if (lane < 16) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 10; ++q) w = lane == q ? t.v[q] : w;
        d[lane] = w;
    }
}
// ten row limbs (any row magnitude <= 16: limbs < 2^31) -> fe26 of magnitude <= 2
__device__ __forceinline__ void fe26_from_row(fe26& r, const uint32_t* l) {
    using namespace f26;
    uint64_t t = 0;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        t += l[q];
        r.v[q] = static_cast<uint32_t>(t) & M26;
        t >>= 26;
    }
    // bits from 2^256 up: x 2^256 = x 977 + x 2^32 (mod p)
    const uint64_t x = (r.v[9] >> 22) + (t << 4);
    r.v[9] &= M22;
    uint64_t u = r.v[0] + x * 977u;
    r.v[0] = static_cast<uint32_t>(u) & M26;
    u = (u >> 26) + r.v[1] + (x << 6);
    r.v[1] = static_cast<uint32_t>(u) & M26;
#pragma unroll
    for (int q = 2; q < 9; ++q) {
        u = (u >> 26) + r.v[q];
        r.v[q] = static_cast<uint32_t>(u) & M26;
    }
    r.v[9] += static_cast<uint32_t>(u >> 26);
    F26_SETM(r, 2);
}
__device__ __forceinline__ void jac_from_row(Jac26& P, const uint32_t (*src)[16], bool inf) {
    fe26_from_row(P.X, src[0]);
    fe26_from_row(P.Y, src[1]);
    fe26_from_row(P.Z, src[2]);
    P.inf = inf;
}

}  // namespace

template <class IO>
__global__ __launch_bounds__(256, 1) void recover_row_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                             int tab_bits) {
    __shared__ RowLds S;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const uint64_t i = blockIdx.x;  // one signature per workgroup (the grid is n)
    if (threadIdx.x < 3) S.post[threadIdx.x] = 0u;
    __syncthreads();
    fe r, s;
    uint32_t v = 0;
    const bool ok = io.rsv(i, r, s, v);
    // ---------------------------------------------------------------- phase A
    if (wave == 3) {
        fe e;
        io.template digest<KECCAK256>(i, e);
        reduce_once(e, ParamN1::M);
        put8(S.e, e, lane);
        row_post(&S.post[0]);
        row_wait(&S.post[1]);
        fe u1;
        get8(u1, S.u1);
        Jac26 G;
        if (tab_bits == kWideBits) comb_mul26<kWideBits>(G, u1, tab);
        else comb_mul26<8>(G, u1, tab);
        fe X, Y, Z;
        fe26_to_fe(X, G.X);
        fe26_to_fe(Y, G.Y);
        fe26_to_fe(Z, G.Z);
        put8(S.g[0], X, lane);
        put8(S.g[1], Y, lane);
        put8(S.g[2], Z, lane);
        if (lane == 0) S.ginf = G.inf ? 1u : 0u;
    } else if (wave == 0) {
        fe rr, ss;
        fe_copy(rr, r);
        fe_copy(ss, s);
        if (!ok) {  // keep the scalar arithmetic well defined (the verdict is already false)
            fe_zero(rr);
            rr.v[0] = 1;
            fe_zero(ss);
        }
        fe rm, rinv;
        FieldN1::from_plain(rm, rr);
        FieldInv<FieldN1>::inv_pipe(rinv, rm);
        row_wait(&S.post[0]);
        fe e, u1, u2, k1, k2;
        get8(e, S.e);
        FieldN1::mul(u1, e, rinv);
        FieldN1::neg(u1, u1);
        FieldN1::mul(u2, ss, rinv);
        bool neg1, neg2;
        glv_split(k1, neg1, k2, neg2, u2);
        put8(S.u1, u1, lane);
        if (lane < 4) {
            S.k[0][lane] = k1.v[lane];
            S.k[1][lane] = k2.v[lane];
        }
        if (lane == 0) S.kflags = (ok ? 1u : 0u) | (neg1 ? 4u : 0u) | (neg2 ? 8u : 0u);
        row_post(&S.post[1]);
    } else {
        fe x;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        fe26 X, w, t, seven;
        fe26_from_fe(X, x);
        fe26_sqr(t, X);
        fe26_mul(w, t, X);
        fe26_set_small(seven, 7u);
        fe26_add(w, w, seven);  // w = x^3 + 7 (m 2)
        if (wave == 2) {
            fe26 y, ny;
            fe26_sqrt_cand(y, w);
            fe26_sqr(t, y);
            fe26_sub<3>(t, t, w);
            okr = okr && fe26_is_zero(t);
            fe26_normalize(y);
            fe26_neg<2>(ny, y);
            fe26_normalize(ny);
            fe26_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            fe yw;
            fe26_to_fe(yw, y);
            put8(S.ys, yw, lane);
            if (lane == 0) S.rflag = okr ? 2u : 0u;
        } else {
            Aff26 R, A[8];
            fe26_mul(R.x, w, X);  // w x
            fe26_sqr(R.y, w);     // w^2
            fe26 Zc, beta;
            {
                Jac26 T[8];
                multiples8_26(T, R);
                coz_table26(A, Zc, T);
            }
            fe26_const(beta, kGlvBeta);
#pragma unroll 1
            for (int j = 0; j < 8; ++j) {
                fe26 bx;
                fe26_mul(bx, A[j].x, beta);
                put_limbs(S.tab[j][0], A[j].x, lane);
                put_limbs(S.tab[j][1], A[j].y, lane);
                put_limbs(S.tab[j][2], bx, lane);
            }
            fe zw;
            fe26_to_fe(zw, Zc);
            put8(S.zc, zw, lane);
            row_post(&S.post[2]);
        }
    }
    // ---------------------------------------------------------------- phase C: the GLV chains on the rows
    if (wave < 2) {
        row_wait(&S.post[1]);
        row_wait(&S.post[2]);
        const frow::Lane L(lane);
        fe k;
        fe_zero(k);
#pragma unroll
        for (int q = 0; q < 4; ++q) k.v[q] = __builtin_amdgcn_readfirstlane(S.k[wave][q]);
        const uint32_t kf = __builtin_amdgcn_readfirstlane(S.kflags);
        const bool neg = (kf & (wave == 0 ? 4u : 8u)) != 0u;
        frow::Pt acc{0u, 0u, 0u};
        const bool fin = frow::glv_chain(acc, k, neg, wave == 1, &S.tab[0][0][0], L);
        if (lane < 16) {
            S.res[wave][0][lane] = acc.X;
            S.res[wave][1][lane] = acc.Y;
            S.res[wave][2][lane] = acc.Z;
        }
        if (lane == 0) S.cinf[wave] = fin ? 0u : 1u;
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase D (wave 0, one lane's work)
    if (wave == 0) {
        Jac26 P0, P1, Q, G, Rq;
        jac_from_row(P0, S.res[0], S.cinf[0] != 0u);
        jac_from_row(P1, S.res[1], S.cinf[1] != 0u);
        CurveK1x::add(Q, P0, P1);  // on the co-Z curve of E_w
        fe zw, yw;
        get8(zw, S.zc);
        get8(yw, S.ys);
        fe26 zc, y;
        fe26_from_fe(zc, zw);
        fe26_from_fe(y, yw);
        fe26_mul(zc, zc, y);
        fe26_mul(Q.Z, Q.Z, zc);  // (X, Y, Z Zc y) on E
        {
            fe X, Y, Z;
            get8(X, S.g[0]);
            get8(Y, S.g[1]);
            get8(Z, S.g[2]);
            fe26_from_fe(G.X, X);
            fe26_from_fe(G.Y, Y);
            fe26_from_fe(G.Z, Z);
            G.inf = S.ginf != 0u;
        }
        CurveK1x::add(Rq, Q, G);
        const bool ok2 = ((S.kflags | S.rflag) & 3u) == 3u && !Rq.inf;
        fe z, zi, ax, ay;
        fe26_to_fe(z, Rq.Z);
        FieldInv<FieldK1>::inv_pipe(zi, z);
        fe26 zi26, zi2, zi3, AX, AY;
        fe26_from_fe(zi26, zi);
        fe26_sqr(zi2, zi26);
        fe26_mul(AX, Rq.X, zi2);
        fe26_mul(zi3, zi2, zi26);
        fe26_mul(AY, Rq.Y, zi3);
        fe26_to_fe(ax, AX);
        fe26_to_fe(ay, AY);
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (ok2 && io.want_addr()) keccak_address(ad, ax, ay);
        if (lane == 0) io.finish(i, ok2, ad, &ax, &ay);
    }
}

template <class IO>
int launch_recover_row(const IO& io, uint64_t n, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits = 8;
    const int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL(recover_row_kernel<IO>, dim3(static_cast<unsigned>(n)), dim3(256), 0, st, io, n, k1, bits);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
template int launch_recover_row<TxIO>(const TxIO&, uint64_t, hipStream_t);
template int launch_recover_row<SigIO>(const SigIO&, uint64_t, hipStream_t);
template int launch_recover_row<EcrecIO>(const EcrecIO&, uint64_t, hipStream_t);

}  // namespace bcosgpu
