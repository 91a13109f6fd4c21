// sm3probe.hip -- lone-wave latency of one SM3 compression four ways: W in registers (sm3_compress),
// sm3_msg over a 512-byte node held in LDS, and over the same node in global memory (AlignedReader),
// in core cycles (s_memtime) and 10 ns ticks (s_memrealtime); and from a block expanded beforehand into
// LDS (sm3_x.h sm3_compress_x, the Merkle kernels' latency-bound levels); with 1 or 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../csrc/hash_device.h"
#include "../csrc/sm3_x.h"
using namespace bcosgpu;

__global__ __launch_bounds__(128) void probe(const uint8_t* g, uint64_t* out, int reps) {
    __shared__ uint32_t buf[2][128];
    __shared__ uint4 wx[2][17];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int q = lane; q < 128; q += 64) buf[w][q] = reinterpret_cast<const uint32_t*>(g)[q] + w;
    __syncthreads();
    uint32_t V[8], W[16], d[8];
    for (int i = 0; i < 8; ++i) V[i] = g[i] + lane;
    for (int i = 0; i < 16; ++i) W[i] = g[8 + i] * 3u + lane;
    uint64_t c0 = clock64(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < reps; ++r) sm3_compress(V, W);
    uint64_t c1 = clock64(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = V[0] ^ V[7];
    if (lane == 0) {
        for (int r = 0; r < reps; ++r) {
            sm3_msg(AlignedReader(reinterpret_cast<const uint8_t*>(&buf[w][0]) + (acc & 4u), 512u - 64u), 512u - 64u, d);
            acc += d[0];
        }
    }
    uint64_t c2 = clock64(), r2 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        for (int r = 0; r < reps; ++r) {
            sm3_msg(AlignedReader(g + 64 * w + (acc & 4u), 512u - 64u), 512u - 64u, d);
            acc += d[0];
        }
    }
    uint64_t c3 = clock64(), r3 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        uint32_t B[16];
        for (int i = 0; i < 16; ++i) B[i] = buf[w][i] ^ acc;
        sm3_expand_block(B, reinterpret_cast<uint32_t*>(&wx[w][0]));
    }
    __syncthreads();
    uint64_t c4 = clock64();
    for (int r = 0; r < reps; ++r) sm3_compress_x(V, reinterpret_cast<const uint32_t*>(&wx[w][0]));
    uint64_t c5 = clock64();
    if (lane == 0) {
        uint64_t* o = out + 12 * (blockIdx.x * 2 + w);
        o[0] = (c1 - c0) / reps; o[1] = (r1 - r0) * 10 / reps;
        o[2] = (c2 - c1) / (8 * reps); o[3] = (r2 - r1) * 10 / (8 * reps);  // 448 B + padding = 8 compressions
        o[4] = (c3 - c2) / (8 * reps); o[5] = (r3 - r2) * 10 / (8 * reps);
        o[6] = acc ^ V[0];
        o[7] = (c5 - c4) / reps;
    }
}

int main() {
    uint8_t* g;
    uint64_t* o;
    if (hipMalloc(&g, 4096) != hipSuccess) return 77;
    (void)hipMemset(g, 0x5a, 4096);
    (void)hipMalloc(&o, 8 * 12 * 4);
    uint64_t h[24];  // 12 words per wave; wave 0's
    for (int waves : {1, 2}) {  // one wave, or two waves of one workgroup (the same SIMD or not: the dispatcher decides)
        hipLaunchKernelGGL(probe, dim3(1), dim3(64 * waves), 0, 0, g, o, 20);
        (void)hipDeviceSynchronize();
        hipLaunchKernelGGL(probe, dim3(1), dim3(64 * waves), 0, 0, g, o, 20);
        (void)hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
        printf("{\"waves\": %d, \"compress_regs\": [%llu cyc, %llu ns], \"per_compression_lds_msg\": [%llu, %llu], "
               "\"per_compression_global_msg\": [%llu, %llu], \"compress_x_lds_expanded\": %llu}\n", waves,
               (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3],
               (unsigned long long)h[4], (unsigned long long)h[5], (unsigned long long)h[7]);
    }
    return 0;
}
