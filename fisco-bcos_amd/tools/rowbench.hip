// rowbench.hip -- cycles per dependent field product: the ROW product of csrc/fe_row.h (one element over
// a 16-lane DPP row, one column per lane) against the one-lane fe26 asm product every kernel runs.
//
// One wave; every row (or lane, for fe26) runs its own chain of N dependent products x <- x * y
// (mode mul) or x <- x^2 (mode sqr).  Prints clock64 cycles per product (lane 0, best of 5) and checks
// (1) every chain's end value against fe26's host products, (2) after EVERY row product, lanes 10..15
// hold 0 and every limb is under the bound fe_row.h states, (3) the DPP moves' lane mapping on a
// pattern.  Usage: rowbench [N]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../csrc/fe26.h"
#include "../csrc/fe_row.h"

using namespace bcosgpu;

constexpr uint32_t kBound = (1u << 26) + (1u << 16);

// MODE 0: fe26 mul (one lane per chain), 1: fe26 sqr, 2: row mul, 3: row sqr, 4 / 5: the SM2 row product /
// square (fe_row.h mul_sm2); CHECK: bound checks
template <int MODE, bool CHECK>
__global__ __launch_bounds__(64) void chain_kernel(const uint32_t* __restrict__ seed, int n, uint32_t* __restrict__ out,
                                                   unsigned long long* __restrict__ cyc, uint32_t* __restrict__ bad) {
    const int lane = threadIdx.x;
    const int k = lane & 15, row = lane >> 4;
    uint32_t flags = 0;
    if constexpr (MODE < 2) {
        fe26 x, y;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            x.v[i] = seed[(lane * 20 + i) & 255] & f26::M26;
            y.v[i] = seed[(lane * 20 + 10 + i) & 255] & f26::M26;
        }
        x.v[9] &= f26::M22;
        y.v[9] &= f26::M22;
        __syncthreads();
        const unsigned long long t0 = clock64();
#pragma unroll 1
        for (int j = 0; j < n; ++j) {
            if constexpr (MODE == 0) fe26_mul(x, x, y);
            else fe26_sqr(x, x);
        }
        const unsigned long long t1 = clock64();
        fe26_normalize(x);
#pragma unroll
        for (int i = 0; i < 10; ++i) out[lane * 10 + i] = x.v[i];
        if (lane == 0) *cyc = t1 - t0;
    } else {
        // row r runs the chain of lane r of the one-lane modes
        uint32_t x = k < 10 ? seed[(row * 20 + k) & 255] & f26::M26 : 0u;
        uint32_t y = k < 10 ? seed[(row * 20 + 10 + k) & 255] & f26::M26 : 0u;
        if (k == 9) {
            x &= f26::M22;
            y &= f26::M22;
        }
        const frow::Lane L(lane);
        const frow::Sm2Lane C(L);
        __syncthreads();
        const unsigned long long t0 = clock64();
#pragma unroll 1
        for (int j = 0; j < n; ++j) {
            if constexpr (MODE == 2) x = frow::mul(x, y, L);
            else if constexpr (MODE == 3) x = frow::sqr(x, L);
            else if constexpr (MODE == 4) x = frow::mul_sm2(x, y, L, C);
            else x = frow::mul_sm2(x, x, L, C);
            if constexpr (CHECK) flags |= (k >= 10 && x != 0u) | (x > kBound ? 2u : 0u);
        }
        const unsigned long long t1 = clock64();
        if (k < 10) out[row * 10 + k] = x;
        if (lane == 0) *cyc = t1 - t0;
        if (CHECK && flags) atomicOr(bad, flags);
    }
}

// lane mapping of the DPP helpers: out[c * 64 + lane] for the helpers in order
__global__ __launch_bounds__(64) void dpp_probe(uint32_t* __restrict__ out) {
    const uint32_t v = 100u + threadIdx.x;
    const int l = threadIdx.x;
    out[0 * 64 + l] = frow::shl<10>(v);
    out[1 * 64 + l] = frow::shr<1>(v);
    out[2 * 64 + l] = frow::shr<6>(v);
    out[3 * 64 + l] = frow::ror<1>(v);
    out[4 * 64 + l] = frow::ror<2>(v);
    out[5 * 64 + l] = frow::bcast<7>(v);
}

// host SM2 reference: x * y mod p over 64-bit words, the 512-bit product folded by 2^256 = 2^224 + 2^96 -
// 2^64 + 1 until it fits 256 bits, then p subtracted while >= p
typedef unsigned __int128 u128;
static const uint64_t kP2[4] = {0xffffffffffffffffull, 0xffffffff00000000ull, 0xffffffffffffffffull,
                                0xfffffffeffffffffull};
static bool ge_p2(const uint64_t a[4]) {
    for (int i = 3; i >= 0; --i)
        if (a[i] != kP2[i]) return a[i] > kP2[i];
    return true;
}
static void sub_p2(uint64_t a[4]) {
    u128 b = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 d = (u128)a[i] - kP2[i] - (uint64_t)b;
        a[i] = (uint64_t)d;
        b = (d >> 64) ? 1 : 0;
    }
}
static void sm2_mulmod(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t t[9] = {0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a[i] * b[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    // fold t[4..8] * 2^256 repeatedly: h * (2^224 + 2^96 - 2^64 + 1) as signed 128-bit columns
    for (int rep = 0; rep < 24; ++rep) {
        uint64_t h[5] = {t[4], t[5], t[6], t[7], t[8]};
        if (!(h[0] | h[1] | h[2] | h[3] | h[4])) break;
        __int128 acc[10] = {0};
        for (int i = 0; i < 4; ++i) acc[i] = t[i];
        // h * 2^224: 2^224 = 2^(3*64 + 32)
        for (int i = 0; i < 5; ++i) {
            acc[i] += (__int128)h[i];                                // + h
            acc[i + 1] -= (__int128)h[i];                            // - h 2^64
            acc[i + 1] += (__int128)(h[i] << 32);                    // + h 2^96 = h 2^32 << 64
            acc[i + 2] += (__int128)(h[i] >> 32);
            acc[i + 3] += (__int128)(h[i] << 32);                    // + h 2^224 = h 2^32 << 192
            acc[i + 4] += (__int128)(h[i] >> 32);
        }
        __int128 c = 0;
        for (int i = 0; i < 9; ++i) {
            c += acc[i];
            t[i] = (uint64_t)c;
            c >>= 64;  // arithmetic (floor) shift
        }
    }
    uint64_t v[4] = {t[0], t[1], t[2], t[3]};
    while (ge_p2(v)) sub_p2(v);
    for (int i = 0; i < 4; ++i) r[i] = v[i];
}
static void limbs_to_p2(uint64_t r[4], const uint32_t* l) {  // sum l_k 2^(26k) mod p (l_k < 2^31)
    uint64_t t[9] = {0};
    for (int k = 0; k < 10; ++k) {
        const int bit = 26 * k;
        u128 v = (u128)l[k] << (bit & 63);
        for (int w = bit >> 6; v && w < 9; ++w) {
            const u128 s = (u128)t[w] + (uint64_t)v;
            t[w] = (uint64_t)s;
            v = (v >> 64) + (s >> 64);
        }
    }
    const uint64_t one[4] = {1, 0, 0, 0};
    uint64_t lo[4] = {t[0], t[1], t[2], t[3]}, hi[4] = {t[4], 0, 0, 0}, p256[4], a[4], b[4];
    // value = lo + hi * 2^256 with hi < 2^5: hi * (2^256 mod p) + lo, through sm2_mulmod
    const uint64_t two256[4] = {1, 0xffffffffull, 0, 0x100000000ull};  // 2^256 mod p
    sm2_mulmod(p256, hi, two256);
    sm2_mulmod(a, lo, one);
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (u128)a[i] + p256[i];
        b[i] = (uint64_t)c;
        c >>= 64;
    }
    if (c || ge_p2(b)) sub_p2(b);
    for (int i = 0; i < 4; ++i) r[i] = b[i];
}

static int probe_errors(const uint32_t* o) {
    int e = 0;
    for (int l = 0; l < 64; ++l) {
        const int r = l & ~15, i = l & 15;
        const uint32_t want[6] = {i + 10 < 16 ? 100u + l + 10 : 0u, i >= 1 ? 100u + l - 1 : 0u, i >= 6 ? 100u + l - 6 : 0u,
                                  100u + r + ((i + 15) & 15), 100u + r + ((i + 14) & 15), 100u + r + 7};
        for (int c = 0; c < 6; ++c) e += o[c * 64 + l] != want[c];
    }
    return e;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    uint32_t hseed[256];
    for (int i = 0; i < 256; ++i) hseed[i] = 0x9E3779B9u * (i + 1) ^ (0x85EBCA6Bu >> (i & 7));
    uint32_t *dseed, *dout, *dbad, *dprobe;
    unsigned long long* dcyc;
    (void)hipMalloc(&dseed, sizeof(hseed));
    (void)hipMalloc(&dout, 640 * 6 * 4);
    (void)hipMalloc(&dcyc, 8 * 30);
    (void)hipMalloc(&dbad, 4);
    (void)hipMalloc(&dprobe, 6 * 64 * 4);
    (void)hipMemset(dbad, 0, 4);
    (void)hipMemcpy(dseed, hseed, sizeof(hseed), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dpp_probe, dim3(1), dim3(64), 0, 0, dprobe);
    // checked pass (bounds after every product), then timed passes
    hipLaunchKernelGGL((chain_kernel<2, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1280, dcyc, dbad);
    hipLaunchKernelGGL((chain_kernel<3, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1920, dcyc, dbad);
    hipLaunchKernelGGL((chain_kernel<4, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 2560, dcyc, dbad);
    hipLaunchKernelGGL((chain_kernel<5, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 3200, dcyc, dbad);
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL((chain_kernel<0, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout, dcyc + 4 * rep, dbad);
        hipLaunchKernelGGL((chain_kernel<1, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 640, dcyc + 4 * rep + 1, dbad);
        hipLaunchKernelGGL((chain_kernel<2, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1280, dcyc + 4 * rep + 2, dbad);
        hipLaunchKernelGGL((chain_kernel<3, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1920, dcyc + 4 * rep + 3, dbad);
        hipLaunchKernelGGL((chain_kernel<4, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 2560, dcyc + 20 + 2 * rep, dbad);
        hipLaunchKernelGGL((chain_kernel<5, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 3200, dcyc + 21 + 2 * rep, dbad);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    unsigned long long hc[30];
    uint32_t ho[3840], hbad, hprobe[384];
    (void)hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hbad, dbad, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hprobe, dprobe, sizeof(hprobe), hipMemcpyDeviceToHost);
    double best[6] = {1e30, 1e30, 1e30, 1e30, 1e30, 1e30};
    for (int rep = 0; rep < 5; ++rep) {
        for (int m = 0; m < 4; ++m)
            if (hc[4 * rep + m] / (double)n < best[m]) best[m] = hc[4 * rep + m] / (double)n;
        for (int m = 0; m < 2; ++m)
            if (hc[20 + 2 * rep + m] / (double)n < best[4 + m]) best[4 + m] = hc[20 + 2 * rep + m] / (double)n;
    }
    // host: the chains of lanes 0..3 with fe26's C++ products; the row results normalised like fe26's
    int mism = 0;
    for (int c = 0; c < 4; ++c) {
        fe26 x, y, xs;
        for (int i = 0; i < 10; ++i) {
            x.v[i] = hseed[(c * 20 + i) & 255] & f26::M26;
            y.v[i] = hseed[(c * 20 + 10 + i) & 255] & f26::M26;
        }
        x.v[9] &= f26::M22;
        y.v[9] &= f26::M22;
        fe26_copy(xs, x);
        for (int j = 0; j < n; ++j) {
            fe26_mul(x, x, y);
            fe26_sqr(xs, xs);
        }
        fe26_normalize(x);
        fe26_normalize(xs);
        fe26 rm, rs;
        for (int i = 0; i < 10; ++i) {
            rm.v[i] = ho[1280 + c * 10 + i];
            rs.v[i] = ho[1920 + c * 10 + i];
        }
        fe26_normalize(rm);
        fe26_normalize(rs);
        int e[4] = {0, 0, 0, 0};
        for (int i = 0; i < 10; ++i) {
            e[0] += x.v[i] != ho[c * 10 + i];
            e[1] += xs.v[i] != ho[640 + c * 10 + i];
            e[2] += x.v[i] != rm.v[i];
            e[3] += xs.v[i] != rs.v[i];
        }
        mism += e[0] + e[1] + e[2] + e[3];
        if (e[0] + e[1] + e[2] + e[3])
            fprintf(stderr, "chain %d: limbs differing fe26_mul %d fe26_sqr %d row_mul %d row_sqr %d\n", c, e[0], e[1],
                    e[2], e[3]);
    }
    // SM2 chains of rows 0..3 against the host reference (the seeds as 26-bit limbs, limb 9 cut at 22 bits)
    int sm2_mism = 0;
    for (int c = 0; c < 4; ++c) {
        uint32_t xl[10], yl[10];
        for (int i = 0; i < 10; ++i) {
            xl[i] = hseed[(c * 20 + i) & 255] & f26::M26;
            yl[i] = hseed[(c * 20 + 10 + i) & 255] & f26::M26;
        }
        xl[9] &= f26::M22;
        yl[9] &= f26::M22;
        uint64_t x[4], y[4], xs[4], gm[4], gs[4];
        limbs_to_p2(x, xl);
        limbs_to_p2(y, yl);
        for (int i = 0; i < 4; ++i) xs[i] = x[i];
        for (int j = 0; j < n; ++j) {
            sm2_mulmod(x, x, y);
            sm2_mulmod(xs, xs, xs);
        }
        limbs_to_p2(gm, ho + 2560 + c * 10);
        limbs_to_p2(gs, ho + 3200 + c * 10);
        for (int i = 0; i < 4; ++i) sm2_mism += (gm[i] != x[i]) + (gs[i] != xs[i]);
    }
    mism += sm2_mism;
    if (sm2_mism) fprintf(stderr, "sm2 chains: %d words differ\n", sm2_mism);
    const int perr = probe_errors(hprobe);
    printf("{\"n\": %d, \"cycles_per_product\": {\"fe26_mul\": %.1f, \"fe26_sqr\": %.1f, \"row_mul\": %.1f, "
           "\"row_sqr\": %.1f, \"row_sm2_mul\": %.1f, \"row_sm2_sqr\": %.1f}, \"mismatches\": %d, \"bound_flags\": %u, \"dpp_probe_errors\": %d, \"note\": "
           "\"clock64 deltas of lane 0 over a dependent chain, best of 5; row = one element over a 16-lane row "
           "(csrc/fe_row.h), four chains per wave\"}\n",
           n, best[0], best[1], best[2], best[3], best[4], best[5], mism, hbad, perr);
    return (mism || hbad || perr) ? 1 : 0;
}
