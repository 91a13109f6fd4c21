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
    uint32_t tab[2][8][3][16];  // GLV tables of R' and 2^64 R' on E_w: x, y, beta x (row limbs, magnitude 1)
    uint32_t zc[2][16];         // their co-Z factors Zc, Zc64
    uint32_t zcy[2][16];        // Zc y, Zc64 y (wave 3)
    uint32_t pt[8][3][16];      // phase D: the four chains' points, the four comb partials, then the sums
    uint32_t pinf[8];
    uint32_t slot[4][16];       // per-wave conversion slot (fe_row -> fe26)
    uint32_t k[2][4];           // GLV halves of u2
    uint32_t u1[8], e[8];
    uint32_t kflags;            // wave 0: bit 0 scalars ok, bit 2 neg1, bit 3 neg2
    uint32_t rflag;             // wave 3: R on the curve (bit 1)
    uint32_t post[4];           // 0: e, 1: k / u1, 2: table of R', 3: table of 2^64 R'
    alignas(8) uint32_t msg[16];  // wave 0: the 64-byte public key for the cooperative address Keccak
    InvQueue invq;                // phase D: Z^-1 split over waves 0 (divsteps, f, g) and 1 (d, e)
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
__device__ __forceinline__ uint32_t sgpr(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// modinv_var_split_fg with (f, g) spread over the rows: lane k < 9 of every row holds limb k (signed
// 30-bit form, lanes 9..15 zero), so a batch's (f, g) <- t (f, g) / 2^30 is two lane-parallel rounds
// instead of nine serial limbs: (1) each lane forms u f_k + v g_k (|.| < 2^60.01), keeps bits 0..29 for
// the lane below and bits 30.. (|.| < 2^30.01) itself -- the exact division by 2^30 is the shift down
// by one lane; (2) the sums (< 2^31.01) split once more, their carries (|.| <= 2) one lane up, the top
// lane keeping its whole signed value.  Limbs stay in [-2, 2^30 + 2) below the top, so the next
// products stay < 2^61.  f0, g0 for the divsteps are limb 0 + 2^30 limb 1 (mod 2^32); g == 0 is tested
// as all limbs zero (a redundant zero only costs further batches, which are exact no-ops), and f's sign
// at the end (f = +-1) from its low word.
__device__ __forceinline__ int32_t inv_fg_rows(const fe& x, const ModInfo30& mi, InvQueue& q, int lane) {
    const int k = lane & 15;
    const uint32_t in9 = frow::mask_if(k < 9), below8 = frow::mask_if(k < 8), top = frow::mask_if(k == 8);
    S30 gs;
    fe_to_s30(gs, x);
    int32_t f = 0, g = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {  // lane k takes limb k (constant indices: no scratch)
        f = k == i ? mi.m[i] : f;
        g = k == i ? gs.v[i] : g;
    }
    f = static_cast<int32_t>(static_cast<uint32_t>(f) & in9);
    g = static_cast<int32_t>(static_cast<uint32_t>(g) & in9);
    auto low32 = [](int32_t a) {  // limb 0 + 2^30 limb 1 (mod 2^32), uniform
        const uint32_t a0 = __builtin_amdgcn_readlane(static_cast<uint32_t>(a), 0);
        const uint32_t a1 = __builtin_amdgcn_readlane(static_cast<uint32_t>(a), 1);
        return a0 + (a1 << 30);
    };
    auto apply = [&](int32_t a, int32_t b, int32_t m1, int32_t m2) {  // (m1 a + m2 b) / 2^30 over the row
        const int64_t c = static_cast<int64_t>(m1) * a + static_cast<int64_t>(m2) * b;
        const uint32_t lo = static_cast<uint32_t>(c) & 0x3fffffffu;
        const int32_t hi = static_cast<int32_t>(c >> 30);
        const int64_t n = static_cast<int64_t>(hi) + frow::shl<1>(lo);  // lane k: bits 30.. of k, 0..29 of k + 1
        const uint32_t lo2 = static_cast<uint32_t>(n) & 0x3fffffffu;
        const uint32_t c2 = static_cast<uint32_t>(static_cast<int32_t>(n >> 30)) & below8;
        const uint32_t keep = frow::bsel(top, static_cast<uint32_t>(n), lo2);
        return static_cast<int32_t>(keep + frow::shr<1>(c2));
    };
    int32_t eta = -1;
#pragma unroll 1
    for (int it = 0; it < 25; ++it) {
        int32_t t[4];
        eta = divsteps_30_var(eta, low32(f), low32(g), t);
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) q.t[it][j] = t[j];
            __hip_atomic_store(&q.n, static_cast<uint32_t>(it + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const int32_t u = __builtin_amdgcn_readfirstlane(t[0]), v = __builtin_amdgcn_readfirstlane(t[1]);
        const int32_t qq = __builtin_amdgcn_readfirstlane(t[2]), r = __builtin_amdgcn_readfirstlane(t[3]);
        const int32_t fn = apply(f, g, u, v), gn = apply(f, g, qq, r);
        f = fn;
        g = gn;
        if (__builtin_amdgcn_ballot_w64(g != 0) == 0) break;
    }
    if (lane == 0) __hip_atomic_store(&q.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return low32(f) == 1u ? 0 : -1;  // f = +-1
}

}  // namespace

// workgroup-0 phase stamps (s_memtime) per wave for tools/rowphase.hip: 0 start, 1 phase-A work done,
// 2 chain done, 6 comb partial done, 3 end; wave 0: 4 / 5 around the affine inversion
#ifdef BCOSGPU_ROW_TIMING
__device__ uint64_t g_row_t[4][8];
#define ROW_T(k) \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_row_t[threadIdx.x >> 6][k] = clock64()
#else
#define ROW_T(k) ((void)0)
#endif

// MODE kRowRecover: public-key recovery (SigIO, TxIO, EcrecIO).  MODE kRowVerify: libsecp256k1
// ecdsa_verify with a KNOWN key P (KeyIO, Secp256k1Crypto.cpp:51-63 for a sealer's unregistered key):
// Q = (e / s) G + (r / s) P, accept iff x(Q) = r (mod n) -- s^-1 instead of r^-1, the tables of P and
// 2^64 P (no square root, no E_w), and the projective x-check instead of the inversion and the address.
enum { kRowRecover = 0, kRowVerify = 1 };
template <int MODE, class IO>
__global__ __launch_bounds__(256, 1) void recover_row_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                             int tab_bits) {
    constexpr bool kVer = MODE == kRowVerify;
    __shared__ RowLds S;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const frow::Lane L(lane);
    const frow::FK1 fk{L};
    uint32_t* const slot = S.slot[wave];
    const uint64_t i = blockIdx.x;  // one signature per workgroup (the grid is n)
    ROW_T(0);
    if (threadIdx.x < 4) S.post[threadIdx.x] = 0u;
    if (threadIdx.x == 0) invq_reset(S.invq);
    __syncthreads();
    fe r, s, kx, ky;
    uint32_t v = 0;
    // every lane parses the same signature: the verdict bits are made wave-uniform (SGPRs), so no branch
    // below depends on a lane's value (a row operation under a partial EXEC would misread its rows)
    bool okp;
    if constexpr (kVer) {
        io.key_rs(i, r, s, kx, ky);
        okp = fe_lt_k(kx, FieldK1::P) && fe_lt_k(ky, FieldK1::P) && !fe_is_zero_raw(r) && !fe_is_zero_raw(s) &&
              fe_lt_k(r, ParamN1::M) && fe_lt_k(s, kN1HalfPlus);  // low-S (secp256k1_ecdsa_verify)
    } else {
        okp = io.rsv(i, r, s, v);
    }
    const bool ok = sgpr(okp ? 1u : 0u) != 0u;
    v = sgpr(v);
    // ---------------------------------------------------------------- phase A
    if (wave == 0) {  // r^-1, u1, u2, the GLV split (one lane's work)
        // recover: u1 = -e / r, u2 = s / r; verify: u1 = e / s, u2 = r / s
        fe inv_of, other;
        fe_copy(inv_of, kVer ? s : r);
        fe_copy(other, kVer ? r : s);
        if (!ok) {  // keep the scalar arithmetic well defined (the verdict is already false)
            fe_zero(inv_of);
            inv_of.v[0] = 1;
            fe_zero(other);
        }
        fe rm, rinv;
        FieldN1::from_plain(rm, inv_of);
        FieldInv<FieldN1>::inv_var(rinv, rm);  // variable time: every lane holds the same value
        row_wait(&S.post[0]);
        fe e, u1, u2, k1, k2;
        get8(e, S.e);
        FieldN1::mul(u1, e, rinv);
        if (!kVer) FieldN1::neg(u1, u1);
        FieldN1::mul(u2, other, rinv);
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
        if (wave == 1) {
            fe e;
            io.template digest<KECCAK256>(i, e);
            reduce_once(e, ParamN1::M);
            put8(S.e, e, lane);
            row_post(&S.post[0]);
        }
        if constexpr (kVer) {
            if (wave == 3) {  // the chains map to E with Z Zc alone
                row_wait(&S.post[2]);
                row_wait(&S.post[3]);
                if (L.row == 0) {
                    S.zcy[0][L.k] = S.zc[0][L.k];
                    S.zcy[1][L.k] = S.zc[1][L.k];
                }
            } else {  // the key's table (wave 1: P, with its on-curve check; wave 2: 2^64 P)
                fe26 X26, Y26;
                fe26_from_fe(X26, kx);
                fe26_from_fe(Y26, ky);
                uint32_t X = frow::from_fe26(X26, L), Y = frow::from_fe26(Y26, L);
                const uint32_t rhs = frow::mul(frow::sqr(X, L), X, L) + 7u * L.one;
                const bool on = frow::is_zero(frow::sub<2>(frow::sqr(Y, L), rhs, L), slot, L);
                if (!(ok && on)) {  // a valid point for a rejected key (its verdict is already false)
                    fe26 gx, gy;
                    fe26_const(gx, kK1Gx);
                    fe26_const(gy, kK1Gy);
                    X = frow::from_fe26(gx, L);
                    Y = frow::from_fe26(gy, L);
                }
                if (wave == 1 && lane == 0) S.rflag = on ? 2u : 0u;
                frow::Pt P{X, Y, L.one};
                if (wave == 2) {
#pragma unroll 1
                    for (int q = 0; q < 64; ++q) frow::dbl(P, fk);
                }
                fe26 beta26;
                fe26_const(beta26, kGlvBeta);
                frow::build_table(S.tab[wave - 1], S.zc[wave - 1], P, frow::from_fe26(beta26, L), fk);
                row_post(&S.post[wave == 1 ? 2 : 3]);
            }
        } else {
        // x = r (+ n), w = x^3 + 7 and R' = (w x, w^2) on E_w: Y^2 = X^3 + 7 w^3 (a point (X, Y, Z) of E_w
        // is (X, Y, Z y) on E, y = sqrt(w))
        fe x;
        fe_copy(x, r);
        bool okr = ok;
        if (v & 2u) {
            okr = okr && fe_lt_k(r, kK1PminusN);
            fe_add_k(x, r, ParamN1::M);
        }
        fe26 X26;
        fe26_from_fe(X26, x);
        const uint32_t X = frow::from_fe26(X26, L);
        const uint32_t w = frow::mul(frow::sqr(X, L), X, L) + 7u * L.one;  // m 1 + 7 / 2^26
        if (wave == 3) {  // y = sqrt(w) with v's parity, then Zc y and Zc64 y
            const uint32_t yc = frow::sqrt_cand(w, fk);
            const bool square = frow::is_zero(frow::sub<2>(frow::sqr(yc, L), w, L), slot, L);
            okr = okr && square;
            fe26 y, ny;
            frow::to_fe26(y, yc, slot, L);
            fe26_normalize(y);
            fe26_neg<2>(ny, y);
            fe26_normalize(ny);
            fe26_cmov(y, ny, (y.v[0] & 1u) != (v & 1u));
            const uint32_t yr = frow::from_fe26(y, L);
            if (lane == 0) S.rflag = okr ? 2u : 0u;
            row_wait(&S.post[2]);
            row_wait(&S.post[3]);
            uint32_t a, b;
            frow::gather01(frow::mul(frow::sel4(L, S.zc[0][L.k], S.zc[1][L.k], S.zc[1][L.k], S.zc[1][L.k]), yr, L), a,
                           b);
            if (L.row == 0) {
                S.zcy[0][L.k] = a;
                S.zcy[1][L.k] = b;
            }
        } else {  // the GLV table of R' (wave 1) or of 2^64 R' (wave 2)
            uint32_t Rx, Ry;
            frow::gather01(frow::mul(w, frow::sel4(L, X, w, w, w), L), Rx, Ry);
            frow::Pt P{Rx, Ry, L.one};
            if (wave == 2) {
#pragma unroll 1
                for (int q = 0; q < 64; ++q) frow::dbl(P, fk);
            }
            fe26 beta26;
            fe26_const(beta26, kGlvBeta);
            frow::build_table(S.tab[wave - 1], S.zc[wave - 1], P, frow::from_fe26(beta26, L), fk);
            row_post(&S.post[wave == 1 ? 2 : 3]);
        }
        }
    }
    ROW_T(1);
    // ---------------------------------------------------------------- phase C: four 64-bit GLV chains
    // wave 0: low half of k1 on R', 1: low half of k2 on phi(R'), 2 / 3: the high halves on 2^64 R'
    row_wait(&S.post[1]);
    row_wait(&S.post[2]);
    row_wait(&S.post[3]);
    {
        const int kh = wave & 1, part = wave >> 1;
        fe k;
        fe_zero(k);
        k.v[2] = sgpr(S.k[kh][2 * part]);
        k.v[3] = sgpr(S.k[kh][2 * part + 1]);
        const uint32_t kf = sgpr(S.kflags);
        const bool neg = (kf & (kh == 0 ? 4u : 8u)) != 0u;
        frow::Pt acc{0u, 0u, 0u};
        const bool fin = frow::glv_chain<16>(acc, k, neg, kh == 1, &S.tab[part][0][0][0], fk);
        frow::pt_store(S.pt[wave], acc, L);
        if (lane == 0) S.pinf[wave] = fin ? 0u : 1u;
    }
    ROW_T(2);
    // ---------------------------------------------------------------- phase D
    {  // u1 G: this wave's quarter of the comb windows (the additions never meet P = +-Q: a partial sum
       // is an integer multiple of G below the window's own 2^(bits i) G multiples)
        constexpr int kW16 = 256 / kWideBits;
        const int W = tab_bits == kWideBits ? kW16 : 32, bits = tab_bits == kWideBits ? kWideBits : 8;
        const int lo = wave * (W / 4), hi = lo + W / 4;
        frow::Pt g{0u, 0u, 0u};
        bool ginf = true;
#pragma unroll 1
        for (int q = lo; q < hi; ++q) {
            const int bit = q * bits;
            const uint32_t wd = sgpr(S.u1[bit >> 5]);
            const uint32_t b = bits == 16 ? (wd >> (bit & 31)) & 0xffffu : (wd >> (bit & 31)) & 0xffu;
            if (b == 0u) continue;
            const uint32_t* e = tab + (static_cast<size_t>(q) << bits | b) * 16;
            const uint32_t ex = frow::from_words(e, L), ey = frow::from_words(e + 8, L);
            if (ginf) {
                g = frow::Pt{ex, ey, L.one};
                ginf = false;
            } else {
                frow::madd(g, ex, ey, fk);
            }
        }
        frow::pt_store(S.pt[4 + wave], g, L);
        if (lane == 0) S.pinf[4 + wave] = ginf ? 1u : 0u;
    }
    ROW_T(6);
    __syncthreads();
    {  // wave 0: chains 0 + 1 (co-Z curve of R') -> E; wave 1: chains 2 + 3 (of 2^64 R') -> E;
       // waves 2, 3: comb partials 0 + 1, 2 + 3
        frow::Pt P, Q, R;
        bool rinf;
        frow::pt_load(P, S.pt[2 * wave], L);
        frow::pt_load(Q, S.pt[2 * wave + 1], L);
        frow::add_full(R, rinf, P, sgpr(S.pinf[2 * wave]) != 0u, Q, sgpr(S.pinf[2 * wave + 1]) != 0u, slot, fk);
        if (wave < 2 && !rinf) R.Z = frow::mul(R.Z, S.zcy[wave][L.k], L);  // (X, Y, Z Zc y) on E
        frow::pt_store(S.pt[2 * wave], R, L);
        if (lane == 0) S.pinf[2 * wave] = rinf ? 1u : 0u;
    }
    __syncthreads();
    if (wave < 2) {  // wave 0: the R part; wave 1: the G part
        frow::Pt P, Q, R;
        bool rinf;
        frow::pt_load(P, S.pt[4 * wave], L);
        frow::pt_load(Q, S.pt[4 * wave + 2], L);
        frow::add_full(R, rinf, P, sgpr(S.pinf[4 * wave]) != 0u, Q, sgpr(S.pinf[4 * wave + 2]) != 0u, slot, fk);
        frow::pt_store(S.pt[4 * wave], R, L);
        if (lane == 0) S.pinf[4 * wave] = rinf ? 1u : 0u;
    }
    __syncthreads();
    if (wave == 0) {  // Q = R part + G part, affine, address
        frow::Pt P, Q, R;
        bool rinf;
        frow::pt_load(P, S.pt[0], L);
        frow::pt_load(Q, S.pt[4], L);
        frow::add_full(R, rinf, P, sgpr(S.pinf[0]) != 0u, Q, sgpr(S.pinf[4]) != 0u, slot, fk);
        const bool ok2 = ((sgpr(S.kflags) | sgpr(S.rflag)) & 3u) == 3u && !rinf;
        Jac26 Rq;
        frow::to_fe26(Rq.X, R.X, slot, L);
        if constexpr (!kVer) frow::to_fe26(Rq.Y, R.Y, slot, L);
        frow::to_fe26(Rq.Z, R.Z, slot, L);
        if constexpr (kVer) {  // x(Q) = X / Z^2 is r or r + n (when r + n < p): X == c Z^2, projectively
            fe26 z2, c, rhs;
            fe xw, cw, r2;
            fe26_sqr(z2, Rq.Z);
            fe26_from_fe(c, r);
            fe26_mul(rhs, c, z2);
            fe26_to_fe(xw, Rq.X);
            fe26_to_fe(cw, rhs);
            bool match = fe_eq_raw(xw, cw);
            const uint32_t carry = fe_add_k(r2, r, ParamN1::M);
            const bool second = carry == 0u && fe_lt_k(r2, FieldK1::P);
            fe26_from_fe(c, second ? r2 : r);
            fe26_mul(rhs, c, z2);
            fe26_to_fe(cw, rhs);
            match = match || (second && fe_eq_raw(xw, cw));
            if (lane == 0) io.finish(i, ok2 && match, nullptr, nullptr, nullptr);
            return;
        } else {
        fe z, zi, ax, ay;
        fe26_to_fe(z, Rq.Z);
        FieldK1::normalize(z);
        ROW_T(4);
        // Z^-1: divsteps and (f, g) over the rows here, the (d, e) updates on wave 1 (modinv_var_split_de)
        const int32_t fsign = inv_fg_rows(z, kMod30K1P, S.invq, lane);
        modinv_var_split_finish(zi, fsign, kMod30K1P, S.invq);
        ROW_T(5);
        fe26 zi26, zi2, zi3, AX, AY;
        fe26_from_fe(zi26, zi);
        fe26_sqr(zi2, zi26);
        fe26_mul(AX, Rq.X, zi2);
        fe26_mul(zi3, zi2, zi26);
        fe26_mul(AY, Rq.Y, zi3);
        fe26_to_fe(ax, AX);
        fe26_to_fe(ay, AY);
        // the address: Keccak-256 of the 64-byte key over 25 lanes (KeccakCoop: ~60 instead of ~180
        // instructions a round), the whole wave taking part (wave-uniform branch); keccak_address's
        // digest words 3..7 = bytes 12..31 are the high half of Keccak lane 1 and lanes 2, 3
        uint32_t ad[5] = {0, 0, 0, 0, 0};
        if (sgpr(ok2 && io.want_addr() ? 1u : 0u) != 0u) {
            uint32_t m[16];
            fe_to_be_words(m, ax);
            fe_to_be_words(m + 8, ay);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < 16; ++q) S.msg[q] = m[q];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const KeccakCoop kc;
            uint32_t lo, hi;
            kc.hash(reinterpret_cast<const uint8_t*>(S.msg), 64u, lo, hi);
            ad[0] = __builtin_amdgcn_readlane(hi, 1);
            ad[1] = __builtin_amdgcn_readlane(lo, 2);
            ad[2] = __builtin_amdgcn_readlane(hi, 2);
            ad[3] = __builtin_amdgcn_readlane(lo, 3);
            ad[4] = __builtin_amdgcn_readlane(hi, 3);
        }
        if (lane == 0) io.finish(i, ok2, ad, &ax, &ay);
        }
    } else if (!kVer && wave == 1) {  // the (d, e) half of wave 0's Z^-1
        modinv_var_split_de(kMod30K1P, S.invq, lane);
    }
    ROW_T(3);
}

// ------------------------------------------------------------------ SM2 verify on the rows
// SM2Crypto::verify / recover with the key (SM2Crypto.cpp:66-92, sm2_do_verify: fast_sm2.cpp:139-227)
// for the smallest batches: Q = s G + t P (t = r + s mod n), accept iff x(Q) = r - e (mod n), e =
// SM3(Z_A || hash).  SM2 has no endomorphism, so t P is split by bit position, t = t_lo + 2^212 t_hi:
// wave 0 builds the key's table and runs t_lo's 53 radix-16 windows (doublings of 3 product levels for
// a = -3 with Z^2 carried: 15 levels a window), while wave 1 doubles the key 212 times, builds that
// point's table and runs t_hi's 11 windows -- about 830 levels each against 995 for one 256-bit chain;
// both check the key on the curve on the rows.  Wave 3 hashes Z_A and e, wave 2 the key's address, and
// then each takes half of the s G comb windows (the comb entries are FieldP2 Montgomery words: one row
// product by R^-1 each); wave 0 adds the three points with complete additions.  The
// x-check is projective (X == c Z^2), so there is no inversion.  Outputs bit-identical to every other
// SM2 verification kernel (tests/test_gpu_row.py, the kernel-variant tests).
__device__ __constant__ static const uint32_t kSm2RowRinv[16] = {0x4u, 0x3fffe40u, 0x6fffu, 0x3f40000u, 0x2ffffffu,
                                                                 0x0u, 0x3ffffc0u, 0x17ffu, 0x3fb0000u, 0x3fffffu,
                                                                 0x0u, 0x0u, 0x0u, 0x0u, 0x0u, 0x0u};
// t = t_lo + 2^kSm2RowSplit t_hi (the SM2 row kernel's two chains, see there)
constexpr int kSm2RowSplit = 212;
namespace {
struct Sm2RowLds {
    uint32_t tab[2][8][3][16];  // the tables of P and of 2^kSm2RowSplit P: x, y (row limbs, magnitude 1)
    uint32_t zc[2][16];
    uint32_t pt[4][3][16];      // the low chain's point, the two comb halves, the high chain's point
    uint32_t pinf[4];
    uint32_t slot[4][16];
    uint32_t c[2][8];        // c = (r - e) mod n and c + n (canonical words)
    uint32_t cflag, kflag, rflag;
    uint32_t ad[5];
    uint32_t post[3];        // 2: comb half of wave 3
};
}  // namespace

template <class IO>
__global__ __launch_bounds__(256, 1) void sm2_verify_row_kernel(IO io, uint64_t n, const uint32_t* __restrict__ tab,
                                                                int tab_bits) {
    __shared__ Sm2RowLds S;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const frow::Lane L(lane);
    const frow::Sm2Lane C(L);
    const frow::FSM2 f{L, C};
    uint32_t* const slot = S.slot[wave];
    const uint64_t i = blockIdx.x;
    if (threadIdx.x < 3) S.post[threadIdx.x] = 0u;
    __syncthreads();
    fe r, s, px, py, t;
    uint32_t X[8], Y[8];
    const bool parsed = io.sm2_sig(i, r, s, X, Y);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        px.v[q] = X[7 - q];
        py.v[q] = Y[7 - q];
    }
    FieldN2::add(t, r, s);
    const bool okp = parsed && fe_lt_k(px, ParamP2::M) && fe_lt_k(py, ParamP2::M) && !fe_is_zero_raw(r) &&
                     !fe_is_zero_raw(s) && fe_lt_k(r, ParamN2::M) && fe_lt_k(s, ParamN2::M) && !fe_is_zero_raw(t);
    const bool ok = sgpr(okp ? 1u : 0u) != 0u;
    const uint32_t rinv = kSm2RowRinv[L.k];
    // ---------------------------------------------------------------- phase A
    // wave 0 only waits for the key's table (wave 1) and then runs the chain: the hashing the final
    // x-check needs -- e = SM3(Z_A || hash), c = r - e -- runs on wave 3 and the key's address on wave 2,
    // each before its half of the s G comb
    if (wave <= 1) {  // the key on the rows and its curve check, on both waves; then the two chains
        fe26 X26, Y26;
        fe26_from_words(X26, px.v);
        fe26_from_words(Y26, py.v);
        uint32_t Xr = frow::from_fe26(X26, L), Yr = frow::from_fe26(Y26, L);
        const uint32_t b = f.mul(frow::from_words(kSM2B, L), rinv);  // b (FieldP2 words are Montgomery)
        const uint32_t x3 = f.mul(f.mul(Xr, Xr), Xr);
        const uint32_t rhs = f.template sub<4>(x3 + b, frow::mul_int<3>(Xr));  // x^3 - 3x + b   m 6
        const bool on = frow::is_zero_sm2(f.template sub<7>(f.mul(Yr, Yr), rhs), slot, L);
        if (!(ok && on)) {  // a valid point for a rejected key (its verdict is already false)
            uint32_t gx, gy;
            frow::gather01(f.mul(frow::sel4(L, frow::from_words(kSM2Gx, L), frow::from_words(kSM2Gy, L),
                                            frow::from_words(kSM2Gy, L), frow::from_words(kSM2Gy, L)),
                                 rinv),
                           gx, gy);
            Xr = gx;
            Yr = gy;
        }
        if (wave == 1 && lane == 0) S.rflag = on ? 2u : 0u;
        // t = t_lo + 2^kSm2RowSplit t_hi: wave 0 runs t_lo over the table of P, wave 1 first doubles P
        // kSm2RowSplit times (3 levels each) and runs t_hi over the table of that point; the split
        // balances the two (3 levels a doubled bit against 3.75 a chain bit)
        fe tt, k;
#pragma unroll
        for (int q = 0; q < 8; ++q) tt.v[q] = sgpr(ok ? t.v[q] : (q == 0 ? 1u : 0u));
        fe_zero(k);
        constexpr int kw = kSm2RowSplit / 32, kb = kSm2RowSplit % 32;
        static_assert(kw == 6 && kb > 0, "t_hi below takes the bits of words 6 and 7");
        frow::Pt P{Xr, Yr, L.one};
        if (wave == 0) {
#pragma unroll
            for (int q = 0; q < kw; ++q) k.v[q] = tt.v[q];
            k.v[kw] = tt.v[kw] & ((1u << kb) - 1u);
        } else {
            k.v[0] = (tt.v[6] >> kb) | (tt.v[7] << (32 - kb));
            k.v[1] = tt.v[7] >> kb;
            uint32_t zz = L.one;
#pragma unroll 1
            for (int q = 0; q < kSm2RowSplit; ++q) frow::dbl_m3z(P, zz, f);
        }
        frow::build_table<frow::FSM2, false>(S.tab[wave], S.zc[wave], P, 0u, f);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        frow::Pt acc{0u, 0u, 0u};
        const bool fin = frow::sm2_chain(acc, k, &S.tab[wave][0][0][0], S.zc[wave][L.k], slot, f);
        frow::pt_store(S.pt[wave == 0 ? 0 : 3], acc, L);
        if (lane == 0) S.pinf[wave == 0 ? 0 : 3] = fin ? 0u : 1u;
    } else if (wave >= 2) {  // waves 2, 3: the hashing, then s G over half of the comb windows each (no
                             // P = +-Q inside a half)
        if (wave == 3) {  // e, c = r - e (mod n)
            fe h, e, c, c2;
            io.template digest<SM3>(i, h);
            uint32_t eb[8];
            sm2_e(eb, X, Y, h);
#pragma unroll
            for (int q = 0; q < 8; ++q) e.v[q] = eb[7 - q];
            reduce_once(e, ParamN2::M);
            FieldN2::sub(c, r, e);
            const uint32_t carry = fe_add_k(c2, c, ParamN2::M);
            const bool second = carry == 0u && fe_lt_k(c2, ParamP2::M);
            put8(S.c[0], c, lane);
            put8(S.c[1], c2, lane);
            if (lane == 0) {
                S.cflag = second ? 1u : 0u;
                S.kflag = ok ? 1u : 0u;
            }
        } else {  // the address of the key
            uint32_t ad[5] = {0, 0, 0, 0, 0};
            if (io.want_addr()) sm3_address(ad, px, py);
            if (lane < 5) {
                uint32_t a = 0;
#pragma unroll
                for (int q = 0; q < 5; ++q) a = lane == q ? ad[q] : a;
                S.ad[lane] = a;
            }
        }
        const int W = tab_bits == kWideBits ? 256 / kWideBits : 32, bits = tab_bits == kWideBits ? kWideBits : 8;
        const int lo = (wave - 2) * (W / 2), hi = lo + W / 2;
        frow::Pt g{0u, 0u, 0u};
        bool ginf = true;
#pragma unroll 1
        for (int q = lo; q < hi; ++q) {
            const int bit = q * bits;
            uint32_t wd = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) wd = (bit >> 5) == u ? s.v[u] : wd;
            wd = sgpr(wd);
            const uint32_t b = bits == 16 ? (wd >> (bit & 31)) & 0xffffu : (wd >> (bit & 31)) & 0xffu;
            if (b == 0u) continue;
            const uint32_t* e = tab + (static_cast<size_t>(q) << bits | b) * 16;
            uint32_t ex, ey;  // Montgomery -> plain
            frow::gather01(f.mul(frow::sel4(L, frow::from_words(e, L), frow::from_words(e + 8, L),
                                            frow::from_words(e + 8, L), frow::from_words(e + 8, L)),
                                 rinv),
                           ex, ey);
            if (ginf) {
                g = frow::Pt{ex, ey, L.one};
                ginf = false;
            } else {
                frow::madd(g, ex, ey, f);
            }
        }
        frow::pt_store(S.pt[wave - 1], g, L);
        if (lane == 0) S.pinf[wave - 1] = ginf ? 1u : 0u;
        if (wave == 3) {
            row_post(&S.post[2]);
        } else {  // wave 2: the two halves
            row_wait(&S.post[2]);
            frow::Pt Q, R;
            bool rinf;
            frow::pt_load(Q, S.pt[2], L);
            frow::add_full(R, rinf, g, ginf, Q, sgpr(S.pinf[2]) != 0u, slot, f);
            frow::pt_store(S.pt[1], R, L);
            if (lane == 0) S.pinf[1] = rinf ? 1u : 0u;
        }
    }
    __syncthreads();
    if (wave == 0) {  // Q = t_lo P + t_hi 2^kSm2RowSplit P + s G, x(Q) == c or c + n, projectively
        frow::Pt P, Q, R;
        bool rinf;
        frow::pt_load(P, S.pt[0], L);
        frow::pt_load(Q, S.pt[3], L);
        frow::add_full(R, rinf, P, sgpr(S.pinf[0]) != 0u, Q, sgpr(S.pinf[3]) != 0u, slot, f);
        P = R;
        const bool pinf = rinf;
        frow::pt_load(Q, S.pt[1], L);
        frow::add_full(R, rinf, P, pinf, Q, sgpr(S.pinf[1]) != 0u, slot, f);
        const uint32_t z2 = f.mul(R.Z, R.Z);
        fe26 c26;
        fe cw;
        get8(cw, S.c[0]);
        fe26_from_words(c26, cw.v);
        bool match = frow::is_zero_sm2(f.template sub<13>(f.mul(frow::from_fe26(c26, L), z2), R.X), slot, L);
        if (sgpr(S.cflag) != 0u) {
            get8(cw, S.c[1]);
            fe26_from_words(c26, cw.v);
            match = match || frow::is_zero_sm2(f.template sub<13>(f.mul(frow::from_fe26(c26, L), z2), R.X), slot, L);
        }
        const bool ok2 = (sgpr(S.kflag) | sgpr(S.rflag)) == 3u && !rinf && match;
        uint32_t ad[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) ad[q] = ok2 ? S.ad[q] : 0u;
        if (lane == 0) io.finish(i, ok2, ad, &px, &py);
    }
}

template <class IO>
int launch_sm2_verify_row(const IO& io, uint64_t n, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits = 8;
    const int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL(sm2_verify_row_kernel<IO>, dim3(static_cast<unsigned>(n)), dim3(256), 0, st, io, n, sm2, bits);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
template int launch_sm2_verify_row<TxIO>(const TxIO&, uint64_t, hipStream_t);
template int launch_sm2_verify_row<SigIO>(const SigIO&, uint64_t, hipStream_t);
template int launch_sm2_verify_row<KeyIO>(const KeyIO&, uint64_t, hipStream_t);

template <class IO>
int launch_recover_row(const IO& io, uint64_t n, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits = 8;
    const int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL((recover_row_kernel<kRowRecover, IO>), dim3(static_cast<unsigned>(n)), dim3(256), 0, st, io, n,
                       k1, bits);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
int launch_sig_verify_row_secp(const KeyIO& io, uint64_t n, hipStream_t st) {
    if (n == 0) return 0;
    const uint32_t *k1, *sm2;
    int bits = 8;
    const int rc = tables(&k1, &sm2, &bits);
    if (rc) return rc;
    hipLaunchKernelGGL((recover_row_kernel<kRowVerify, KeyIO>), dim3(static_cast<unsigned>(n)), dim3(256), 0, st, io,
                       n, k1, bits);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
template int launch_recover_row<TxIO>(const TxIO&, uint64_t, hipStream_t);
template int launch_recover_row<SigIO>(const SigIO&, uint64_t, hipStream_t);
template int launch_recover_row<EcrecIO>(const EcrecIO&, uint64_t, hipStream_t);

}  // namespace bcosgpu
