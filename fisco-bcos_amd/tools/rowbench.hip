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

// MODE 0: fe26 mul (one lane per chain), 1: fe26 sqr, 2: row mul, 3: row sqr; CHECK: bound checks
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
        __syncthreads();
        const unsigned long long t0 = clock64();
#pragma unroll 1
        for (int j = 0; j < n; ++j) {
            if constexpr (MODE == 2) x = frow::mul(x, y, L);
            else x = frow::sqr(x, L);
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
    (void)hipMalloc(&dout, 640 * 4 * 4);
    (void)hipMalloc(&dcyc, 8 * 4 * 5);
    (void)hipMalloc(&dbad, 4);
    (void)hipMalloc(&dprobe, 6 * 64 * 4);
    (void)hipMemset(dbad, 0, 4);
    (void)hipMemcpy(dseed, hseed, sizeof(hseed), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dpp_probe, dim3(1), dim3(64), 0, 0, dprobe);
    // checked pass (bounds after every product), then timed passes
    hipLaunchKernelGGL((chain_kernel<2, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1280, dcyc, dbad);
    hipLaunchKernelGGL((chain_kernel<3, true>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1920, dcyc, dbad);
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL((chain_kernel<0, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout, dcyc + 4 * rep, dbad);
        hipLaunchKernelGGL((chain_kernel<1, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 640, dcyc + 4 * rep + 1, dbad);
        hipLaunchKernelGGL((chain_kernel<2, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1280, dcyc + 4 * rep + 2, dbad);
        hipLaunchKernelGGL((chain_kernel<3, false>), dim3(1), dim3(64), 0, 0, dseed, n, dout + 1920, dcyc + 4 * rep + 3, dbad);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    unsigned long long hc[20];
    uint32_t ho[2560], hbad, hprobe[384];
    (void)hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hbad, dbad, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hprobe, dprobe, sizeof(hprobe), hipMemcpyDeviceToHost);
    double best[4] = {1e30, 1e30, 1e30, 1e30};
    for (int rep = 0; rep < 5; ++rep)
        for (int m = 0; m < 4; ++m)
            if (hc[4 * rep + m] / (double)n < best[m]) best[m] = hc[4 * rep + m] / (double)n;
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
    const int perr = probe_errors(hprobe);
    printf("{\"n\": %d, \"cycles_per_product\": {\"fe26_mul\": %.1f, \"fe26_sqr\": %.1f, \"row_mul\": %.1f, "
           "\"row_sqr\": %.1f}, \"mismatches\": %d, \"bound_flags\": %u, \"dpp_probe_errors\": %d, \"note\": "
           "\"clock64 deltas of lane 0 over a dependent chain, best of 5; row = one element over a 16-lane row "
           "(csrc/fe_row.h), four chains per wave\"}\n",
           n, best[0], best[1], best[2], best[3], mism, hbad, perr);
    return (mism || hbad || perr) ? 1 : 0;
}
