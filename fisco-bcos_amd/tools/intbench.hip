// intbench.hip -- measures the gfx950 integer-ALU peaks that bound this engine's kernels
// (the roofline denominators in bench.py / DESIGN.md).  Each kernel runs 8 independent
// dependency chains of ONE instruction (inline asm, so exactly that opcode is issued) per lane,
// on 256 CUs x 8 waves/SIMD.  Prints JSON: lane-ops per second for each instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
#define CHAINS 8

#define KERNEL32(NAME, ASM)                                                        \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {    \
        uint32_t x[CHAINS];                                                        \
        const uint32_t c = seed | 1u;                                              \
        for (int k = 0; k < CHAINS; ++k) x[k] = threadIdx.x * 7919u + k + seed;     \
        for (int it = 0; it < ITERS; ++it) {                                       \
            _Pragma("unroll") for (int k = 0; k < CHAINS; ++k) {                   \
                asm volatile(ASM : "+v"(x[k]) : "v"(c));                           \
            }                                                                      \
        }                                                                          \
        uint32_t r = 0;                                                            \
        for (int k = 0; k < CHAINS; ++k) r ^= x[k];                                \
        if (r == 0x12345678u) out[0] = r;                                          \
    }

KERNEL32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL32(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
KERNEL32(k_xor3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
KERNEL32(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERNEL32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL32(k_bfi, "v_bfi_b32 %0, %0, %1, %0")

__global__ __launch_bounds__(256) void k_mad_u64(uint32_t* out, uint32_t seed) {
    uint64_t x[CHAINS];
    const uint32_t c = seed | 1u;
    for (int k = 0; k < CHAINS; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) {
            uint64_t cc;
            uint32_t lo = static_cast<uint32_t>(x[k]);
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x[k]), "=s"(cc) : "v"(lo), "v"(c));
        }
    }
    uint64_t r = 0;
    for (int k = 0; k < CHAINS; ++k) r ^= x[k];
    if (r == 0x12345678u) out[0] = static_cast<uint32_t>(r);
}

__global__ __launch_bounds__(256) void k_add_co(uint32_t* out, uint32_t seed) {
    uint32_t x[CHAINS];
    const uint32_t c = seed | 1u;
    for (int k = 0; k < CHAINS; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) {
            uint64_t cc;
            asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(x[k]), "=s"(cc) : "v"(c));
        }
    }
    uint32_t r = 0;
    for (int k = 0; k < CHAINS; ++k) r ^= x[k];
    if (r == 0x12345678u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_fma_f64(uint32_t* out, uint32_t seed) {
    double x[CHAINS];
    const double c = 1.0000001, d = 1e-9 * seed;
    for (int k = 0; k < CHAINS; ++k) x[k] = threadIdx.x + k;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[k]) : "v"(c), "v"(d));
    }
    double r = 0;
    for (int k = 0; k < CHAINS; ++k) r += x[k];
    if (r == 1234.5) out[0] = 1;
}

typedef void (*kfn)(uint32_t*, uint32_t);

static double run(kfn f, uint32_t* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 3u);  // warm-up
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 3u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double ops = 5.0 * blocks * 256.0 * ITERS * CHAINS;
    return ops / (ms * 1e-3);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 8;  // 8 x 256 threads per CU = 8 waves/SIMD
    struct { const char* name; kfn f; } ks[] = {
        {"v_mad_u64_u32", k_mad_u64}, {"v_mul_lo_u32", k_mul_lo},   {"v_mul_hi_u32", k_mul_hi},
        {"v_mul_u32_u24", k_mul_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_mad_u32_u24", k_mad_u24},
        {"v_add_co_u32", k_add_co},   {"v_bitop3_b32", k_xor3},       {"v_add3_u32", k_add3},
        {"v_alignbit_b32", k_alignbit}, {"v_bfi_b32", k_bfi},       {"v_fma_f64", k_fma_f64}};
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"lane_ops_per_s\": {", p.gcnArchName,
           p.multiProcessorCount, p.clockRate);
    for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i)
        printf("%s\"%s\": %.4e", i ? ", " : "", ks[i].name, run(ks[i].f, out, blocks));
    printf("}}\n");
    return 0;
}
