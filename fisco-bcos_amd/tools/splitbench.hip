// splitbench.hip -- A/B of a LANE-PAIR split secp256k1 field product against the one-lane fe26 product
// (round-4 verdict, item 5: can splitting one 256-bit product over several lanes of a wave shorten the
// serial point chain of the latency kernels?).
//
// One wave, a dependent chain of N products x <- x * y on every lane (or lane pair):
//   asm     fe26_mul_asm / fe26_sqr_asm (fe_asm.h, what every kernel runs), one lane per chain;
//   cxx     the same column / fold algorithm in C++ (fe26.h's host path, compiler-scheduled), one lane;
//   pair    the product split over a lane pair: both lanes hold a and b; the odd lane reverses its
//           operands (A_u = a_{9-u}, B_v = b_{9-v}) so that ONE uniform instruction stream of 55
//           v_mad_u64_u32 gives the even lane the low columns c_0..c_9 and the odd lane the high
//           columns c_18..c_9; the high columns cross to the even lane by DPP swaps (18 dwords), the
//           fold and carries run as in fe26_reduce, and the result is broadcast back to the odd lane
//           (10 DPP moves) for the next product.
// Prints cycles per product (s_memtime deltas of lane 0, median of the wave's repetitions) and checks
// that all three chains end at the same value.  Usage: splitbench [N]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../csrc/fe26.h"

using namespace bcosgpu;

// fe26_reduce's algorithm (fe26.h), kept out of line from the asm path
__device__ __forceinline__ void reduce_cxx(fe26& r, const uint64_t c[19]) { fe26_reduce(r, c); }

__device__ __forceinline__ void mul_cxx(fe26& r, const fe26& a, const fe26& b) {
    uint64_t c[19];
#pragma unroll
    for (int k = 0; k < 19; ++k) {
        uint64_t s = 0;
#pragma unroll
        for (int i = (k < 10 ? 0 : k - 9); i <= (k < 10 ? k : 9); ++i) s += static_cast<uint64_t>(a.v[i]) * b.v[k - i];
        c[k] = s;
    }
    reduce_cxx(r, c);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, false));
}
constexpr int kSwap = 0xB1;   // quad_perm [1, 0, 3, 2]: lane pairs swap
constexpr int kBcast = 0xA0;  // quad_perm [0, 0, 2, 2]: the even lane's value to both

// x * y over the lane pair (odd = lane & 1); r replicated on both lanes
__device__ __forceinline__ void mul_pair(fe26& r, const fe26& a, const fe26& b, bool odd) {
    uint32_t A[10], B[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) {
        A[u] = odd ? a.v[9 - u] : a.v[u];
        B[u] = odd ? b.v[9 - u] : b.v[u];
    }
    uint64_t s[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        uint64_t t = 0;
#pragma unroll
        for (int u = 0; u <= j; ++u) t += static_cast<uint64_t>(A[u]) * B[j - u];
        s[j] = t;
    }
    uint64_t c[19];
#pragma unroll
    for (int j = 0; j < 10; ++j) c[j] = s[j];
#pragma unroll
    for (int k = 10; k < 19; ++k) {  // c_k = the odd lane's s_{18-k}
        const uint64_t v = s[18 - k];
        const uint32_t lo = dpp<kSwap>(static_cast<uint32_t>(v)), hi = dpp<kSwap>(static_cast<uint32_t>(v >> 32));
        c[k] = (static_cast<uint64_t>(hi) << 32) | lo;
    }
    fe26 t;
    reduce_cxx(t, c);
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = dpp<kBcast>(t.v[i]);
}

template <int MODE>
__global__ __launch_bounds__(64) void chain_kernel(const uint32_t* __restrict__ seed, int n, uint32_t* __restrict__ out,
                                                   unsigned long long* __restrict__ cyc) {
    const int lane = threadIdx.x;
    const bool odd = lane & 1;
    const int chain = MODE == 2 ? lane >> 1 : lane;
    fe26 x, y;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        x.v[i] = seed[(chain * 20 + i) & 255] & f26::M26;
        y.v[i] = seed[(chain * 20 + 10 + i) & 255] & f26::M26;
    }
    x.v[9] &= f26::M22;
    y.v[9] &= f26::M22;
    __syncthreads();
    const unsigned long long t0 = clock64();
#pragma unroll 1
    for (int k = 0; k < n; ++k) {
        if constexpr (MODE == 0) fe26_mul(x, x, y);  // fe26_mul_asm on the device
        else if constexpr (MODE == 1) mul_cxx(x, x, y);
        else mul_pair(x, x, y, odd);
    }
    const unsigned long long t1 = clock64();
    fe26_normalize(x);
#pragma unroll
    for (int i = 0; i < 10; ++i) out[lane * 10 + i] = x.v[i];
    if (lane == 0) *cyc = t1 - t0;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    uint32_t hseed[256];
    for (int i = 0; i < 256; ++i) hseed[i] = 0x9E3779B9u * (i + 1) ^ (0x85EBCA6Bu >> (i & 7));
    uint32_t *dseed, *dout;
    unsigned long long* dcyc;
    (void)hipMalloc(&dseed, sizeof(hseed));
    (void)hipMalloc(&dout, 64 * 10 * 4 * 3);
    (void)hipMalloc(&dcyc, 8 * 3 * 5);
    (void)hipMemcpy(dseed, hseed, sizeof(hseed), hipMemcpyHostToDevice);
    double best[3] = {1e30, 1e30, 1e30};
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(chain_kernel<0>, dim3(1), dim3(64), 0, 0, dseed, n, dout, dcyc + 3 * rep);
        hipLaunchKernelGGL(chain_kernel<1>, dim3(1), dim3(64), 0, 0, dseed, n, dout + 640, dcyc + 3 * rep + 1);
        hipLaunchKernelGGL(chain_kernel<2>, dim3(1), dim3(64), 0, 0, dseed, n, dout + 1280, dcyc + 3 * rep + 2);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    unsigned long long hc[15];
    uint32_t ho[1920];
    (void)hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    for (int rep = 0; rep < 5; ++rep)
        for (int m = 0; m < 3; ++m)
            if (hc[3 * rep + m] / (double)n < best[m]) best[m] = hc[3 * rep + m] / (double)n;
    // lanes 0..31 of the one-lane chains equal the pair chains' (pair p = lanes 2p, 2p+1 runs chain p)
    int bad = 0;
    for (int c = 0; c < 32; ++c)
        for (int i = 0; i < 10; ++i) {
            const uint32_t a = ho[c * 10 + i], b = ho[640 + c * 10 + i];
            const uint32_t p0 = ho[1280 + (2 * c) * 10 + i], p1 = ho[1280 + (2 * c + 1) * 10 + i];
            bad += a != b || a != p0 || a != p1;
        }
    printf("{\"n\": %d, \"cycles_per_mul\": {\"asm_one_lane\": %.1f, \"cxx_one_lane\": %.1f, \"pair_split\": %.1f}, "
           "\"mismatches\": %d, \"note\": \"clock64 deltas of lane 0 over a dependent chain, best of 5\"}\n",
           n, best[0], best[1], best[2], bad);
    return bad ? 1 : 0;
}
