// carrybench.hip -- checks, on the GPU, whether 256-bit add-with-carry chains written as VOP3
// v_add_co/v_addc_co with an explicit SGPR-pair carry (no s_nop between dependent steps) produce the
// same results as the compiler's own chains (which it pads with s_nop on gfx950), and times both.
// Used to decide how the field arithmetic's carry chains are written.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    return s;
}

// compiler chain (__builtin_addc), dependent across iterations
__global__ void k_builtin(uint32_t* out, uint32_t seed) {
    uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    uint32_t a[8], b[8];
    for (int i = 0; i < 8; ++i) { a[i] = xs(s); b[i] = xs(s); }
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) { unsigned co; a[i] = __builtin_addc(a[i], b[i], c, &co); c = co; }
        acc += c;
        b[it & 7] ^= a[(it + 3) & 7];
    }
    uint32_t h = acc;
    for (int i = 0; i < 8; ++i) h = h * 31u + a[i];
    out[blockIdx.x * 256 + threadIdx.x] = h;
}

// hand chain: VOP3 with SGPR-pair carry, no wait states between dependent steps
__global__ void k_asm(uint32_t* out, uint32_t seed) {
    uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    uint32_t a[8], b[8];
    for (int i = 0; i < 8; ++i) { a[i] = xs(s); b[i] = xs(s); }
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        uint32_t c;
        uint64_t cc;
        asm volatile(
            "v_add_co_u32_e64 %0, %9, %0, %10\n\t"
            "v_addc_co_u32_e64 %1, %9, %1, %11, %9\n\t"
            "v_addc_co_u32_e64 %2, %9, %2, %12, %9\n\t"
            "v_addc_co_u32_e64 %3, %9, %3, %13, %9\n\t"
            "v_addc_co_u32_e64 %4, %9, %4, %14, %9\n\t"
            "v_addc_co_u32_e64 %5, %9, %5, %15, %9\n\t"
            "v_addc_co_u32_e64 %6, %9, %6, %16, %9\n\t"
            "v_addc_co_u32_e64 %7, %9, %7, %17, %9\n\t"
            "v_addc_co_u32_e64 %8, %9, 0, 0, %9"
            : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
              "=v"(c), "=&s"(cc)
            : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
        acc += c;
        b[it & 7] ^= a[(it + 3) & 7];
    }
    uint32_t h = acc;
    for (int i = 0; i < 8; ++i) h = h * 31u + a[i];
    out[blockIdx.x * 256 + threadIdx.x] = h;
}

// same with VOP2 implicit-VCC carries, no wait states
__global__ void k_asm_vcc(uint32_t* out, uint32_t seed) {
    uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    uint32_t a[8], b[8];
    for (int i = 0; i < 8; ++i) { a[i] = xs(s); b[i] = xs(s); }
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        uint32_t c;
        asm volatile(
            "v_add_co_u32_e32 %0, vcc, %0, %9\n\t"
            "v_addc_co_u32_e32 %1, vcc, %1, %10, vcc\n\t"
            "v_addc_co_u32_e32 %2, vcc, %2, %11, vcc\n\t"
            "v_addc_co_u32_e32 %3, vcc, %3, %12, vcc\n\t"
            "v_addc_co_u32_e32 %4, vcc, %4, %13, vcc\n\t"
            "v_addc_co_u32_e32 %5, vcc, %5, %14, vcc\n\t"
            "v_addc_co_u32_e32 %6, vcc, %6, %15, vcc\n\t"
            "v_addc_co_u32_e32 %7, vcc, %7, %16, vcc\n\t"
            "v_addc_co_u32_e64 %8, s[100:101], 0, 0, vcc"
            : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
              "=v"(c)
            : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
            : "vcc", "s100", "s101");
        acc += c;
        b[it & 7] ^= a[(it + 3) & 7];
    }
    uint32_t h = acc;
    for (int i = 0; i < 8; ++i) h = h * 31u + a[i];
    out[blockIdx.x * 256 + threadIdx.x] = h;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    const int blocks = 2048, n = blocks * 256;
    uint32_t *o1, *o2, *o3;
    (void)hipMalloc(&o1, n * 4);
    (void)hipMalloc(&o2, n * 4);
    (void)hipMalloc(&o3, n * 4);
    kfn ks[3] = {k_builtin, k_asm, k_asm_vcc};
    uint32_t* os[3] = {o1, o2, o3};
    float ms[3];
    long mism[3] = {0, 0, 0};
    uint32_t* h[3];
    for (int r = 0; r < 3; ++r) h[r] = new uint32_t[n];
    for (int seed = 1; seed <= 8; ++seed) {
        for (int v = 0; v < 3; ++v) {
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, os[v], (uint32_t)seed * 977u);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms[v], a, b);
            (void)hipMemcpy(h[v], os[v], n * 4, hipMemcpyDeviceToHost);
        }
        for (int v = 1; v < 3; ++v)
            for (int i = 0; i < n; ++i) mism[v] += h[v][i] != h[0][i];
    }
    printf("{\"chains_checked\": %ld, \"mismatch_sgpr_nonop\": %ld, \"mismatch_vcc_nonop\": %ld, "
           "\"ms_builtin\": %.3f, \"ms_sgpr_nonop\": %.3f, \"ms_vcc_nonop\": %.3f}\n",
           (long)n * ITERS * 8, mism[1], mism[2], ms[0], ms[1], ms[2]);
    return 0;
}
