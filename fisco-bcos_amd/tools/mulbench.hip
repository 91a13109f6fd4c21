// mulbench.hip -- latency vs throughput of the 256-bit field arithmetic on gfx950, measured in
// shader-clock cycles per operation (s_memtime) with 1 and 2 waves per SIMD.  Answers: is a lone
// wave (the C2 / small-batch regime) issue-bound or dependency-latency-bound in FieldK1::mul?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include "../csrc/fe.h"
#include "../csrc/ec.h"
#include "../csrc/ec26.h"

using namespace bcosgpu;
#define ITERS 2000

__device__ __forceinline__ void seed_fe(fe& x, uint32_t s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x.v[i] = s * 2654435761u + i * 40503u + 1u;
    x.v[7] &= 0x7fffffffu;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k_mul(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe x[CHAINS], y;
    seed_fe(y, s + 99);
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) seed_fe(x[c], s + threadIdx.x + c);
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) FieldK1::mul(x[c], x[c], y);
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c].v[0] ^ x[c].v[7];
    if (r == 0x12345678u) out[0] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
__global__ __launch_bounds__(256) void k_fmul(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe x, y;
    seed_fe(y, s + 99);
    seed_fe(x, s + threadIdx.x);
    y.v[7] &= 0x0fffffffu;
    x.v[7] &= 0x0fffffffu;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) F::mul(x, x, y);
    const uint64_t t1 = clock64();
    if ((x.v[0] ^ x.v[7]) == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <class F>
__global__ __launch_bounds__(256) void k_fsqr(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe x;
    seed_fe(x, s + threadIdx.x);
    x.v[7] &= 0x0fffffffu;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) F::sqr(x, x);
    const uint64_t t1 = clock64();
    if ((x.v[0] ^ x.v[7]) == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k_sqr(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) seed_fe(x[c], s + threadIdx.x + c);
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) FieldK1::sqr(x[c], x[c]);
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c].v[0] ^ x[c].v[7];
    if (r == 0x12345678u) out[0] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_dbl(uint64_t* cyc, uint32_t* out, uint32_t s) {
    Jac P;
    seed_fe(P.X, s + threadIdx.x);
    seed_fe(P.Y, s + threadIdx.x + 7);
    seed_fe(P.Z, s + threadIdx.x + 9);
    P.inf = false;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS / 8; ++it) CurveK1::dbl(P, P);
    const uint64_t t1 = clock64();
    if ((P.X.v[0] ^ P.Y.v[3]) == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k_madchain(uint64_t* cyc, uint32_t* out, uint32_t s) {
    uint64_t acc[CHAINS];
    uint32_t c2[CHAINS];
    const uint32_t a = s * 7u + threadIdx.x, b = s ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) { acc[c] = c; c2[c] = 0; }
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS * 8; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) BG_MADC(acc[c], c2[c], a, b);
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= acc[c] ^ c2[c];
    if (r == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// v_mad_u64_u32 without using the carry-out (acc = a*b + acc): the 26-bit-limb accumulation pattern
template <int CHAINS>
__global__ __launch_bounds__(256) void k_madnc(uint64_t* cyc, uint32_t* out, uint32_t s) {
    uint64_t acc[CHAINS];
    const uint32_t a = s * 7u + threadIdx.x, b = s ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = c;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS * 8; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            uint64_t cc;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
        }
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= acc[c];
    if (r == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// 64-bit adds via v_lshl_add_u64 (gfx940+): acc = (x << 1) + acc
template <int CHAINS>
__global__ __launch_bounds__(256) void k_lshladd(uint64_t* cyc, uint32_t* out, uint32_t s) {
    uint64_t acc[CHAINS];
    const uint64_t b = s ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS * 8; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_lshl_add_u64 %0, %1, 1, %0" : "+v"(acc[c]) : "v"(b));
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= acc[c];
    if (r == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// plain 32-bit adds
template <int CHAINS>
__global__ __launch_bounds__(256) void k_add(uint64_t* cyc, uint32_t* out, uint32_t s) {
    uint32_t x[CHAINS];
    const uint32_t b = s ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = c + threadIdx.x;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS * 8; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x[c]) : "v"(b));
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c];
    if (r == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// v_mul_lo + v_mul_hi pairs (32x32 -> 64 without mad)
template <int CHAINS>
__global__ __launch_bounds__(256) void k_mulpair(uint64_t* cyc, uint32_t* out, uint32_t s) {
    uint32_t x[CHAINS], y[CHAINS];
    const uint32_t b = s ^ 0x9e3779b9u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) { x[c] = c + threadIdx.x; y[c] = c; }
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS * 8; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            asm volatile("v_mul_lo_u32 %0, %1, %2\n\tv_mul_hi_u32 %1, %1, %2" : "=&v"(y[c]), "+v"(x[c]) : "v"(b));
        }
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c] ^ y[c];
    if (r == 0x12345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}


__device__ __forceinline__ void seed_fe26(fe26& x, uint32_t s) {
#pragma unroll
    for (int i = 0; i < 10; ++i) x.v[i] = (s * 2654435761u + i * 40503u + 1u) & 0x3ffffffu;
    x.v[9] &= 0x3fffffu;
}
template <int CHAINS>
__global__ __launch_bounds__(256) void k_f26mul(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe26 x[CHAINS], y;
    seed_fe26(y, s + 99);
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) seed_fe26(x[c], s + threadIdx.x + c);
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) fe26_mul(x[c], x[c], y);
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c].v[0] ^ x[c].v[7];
    if (r == 0x00345678u) out[0] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int CHAINS>
__global__ __launch_bounds__(256) void k_f26sqr(uint64_t* cyc, uint32_t* out, uint32_t s) {
    fe26 x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) seed_fe26(x[c], s + threadIdx.x + c);
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) fe26_sqr(x[c], x[c]);
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c].v[0] ^ x[c].v[7];
    if (r == 0x00345678u) out[0] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ __launch_bounds__(256) void k_f26dbl(uint64_t* cyc, uint32_t* out, uint32_t s) {
    Jac26 P;
    seed_fe26(P.X, s + threadIdx.x);
    seed_fe26(P.Y, s + threadIdx.x + 7);
    seed_fe26(P.Z, s + threadIdx.x + 9);
    P.inf = false;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS / 8; ++it) CurveK1x::dbl(P, P);
    const uint64_t t1 = clock64();
    if ((P.X.v[0] ^ P.Y.v[3]) == 0x00345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ __launch_bounds__(256) void k_madd(uint64_t* cyc, uint32_t* out, uint32_t s) {
    Jac P;
    Aff Q;
    seed_fe(P.X, s + threadIdx.x);
    seed_fe(P.Y, s + threadIdx.x + 7);
    seed_fe(P.Z, s + threadIdx.x + 9);
    seed_fe(Q.x, s + 3);
    seed_fe(Q.y, s + 5);
    P.inf = false;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS / 8; ++it) CurveK1::madd(P, P, Q);
    const uint64_t t1 = clock64();
    if ((P.X.v[0] ^ P.Y.v[3]) == 0x00345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ __launch_bounds__(256) void k_f26madd(uint64_t* cyc, uint32_t* out, uint32_t s) {
    Jac26 P;
    Aff26 Q;
    seed_fe26(P.X, s + threadIdx.x);
    seed_fe26(P.Y, s + threadIdx.x + 7);
    seed_fe26(P.Z, s + threadIdx.x + 9);
    seed_fe26(Q.x, s + 3);
    seed_fe26(Q.y, s + 5);
    P.inf = false;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS / 8; ++it) CurveK1x::madd(P, P, Q);
    const uint64_t t1 = clock64();
    if ((P.X.v[0] ^ P.Y.v[3]) == 0x00345678u) out[0] = 1;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char* name, K kern, int waves_per_simd, double ops_per_iter, int iters, uint64_t* d_cyc, uint32_t* d_out,
                bool last) {
    const int blocks = 256 * waves_per_simd;  // 4 waves per block, 256 CUs
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_cyc, d_out, 1u);  // warm-up
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_cyc, d_out, 2u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t* h = new uint64_t[blocks];
    hipMemcpy(h, d_cyc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += h[i];
    avg /= blocks;
    delete[] h;
    const double per_op = avg / (iters * ops_per_iter);
    const double lane_ops = double(blocks) * 256 * iters * ops_per_iter / (ms * 1e-3);
    printf("  \"%s_occ%d\": {\"cycles_per_op_per_wave\": %.1f, \"lane_ops_per_s\": %.4e, \"ms\": %.3f}%s\n", name,
           waves_per_simd, per_op, lane_ops, ms, last ? "" : ",");
}

int main() {
    uint64_t* d_cyc;
    uint32_t* d_out;
    hipMalloc(&d_cyc, 4096 * 8);
    hipMalloc(&d_out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("{\"device\": \"%s\", \"clock_khz\": %d,\n", p.gcnArchName, p.clockRate);
    const bool quick = getenv("MULBENCH_QUICK") != nullptr;
    for (int occ = 1; occ <= 4; occ *= 2) {
        if (!quick) {
            run("madnc_chain1", k_madnc<1>, occ, 1, ITERS * 8, d_cyc, d_out, false);
            run("madnc_chain4", k_madnc<4>, occ, 4, ITERS * 8, d_cyc, d_out, false);
            run("lshladd_chain1", k_lshladd<1>, occ, 1, ITERS * 8, d_cyc, d_out, false);
            run("lshladd_chain4", k_lshladd<4>, occ, 4, ITERS * 8, d_cyc, d_out, false);
            run("add_chain1", k_add<1>, occ, 1, ITERS * 8, d_cyc, d_out, false);
            run("add_chain4", k_add<4>, occ, 4, ITERS * 8, d_cyc, d_out, false);
            run("mulpair_chain4", k_mulpair<4>, occ, 4, ITERS * 8, d_cyc, d_out, false);
            run("madc_chain1", k_madchain<1>, occ, 1, ITERS * 8, d_cyc, d_out, false);
            run("madc_chain2", k_madchain<2>, occ, 2, ITERS * 8, d_cyc, d_out, false);
            run("madc_chain4", k_madchain<4>, occ, 4, ITERS * 8, d_cyc, d_out, false);
            run("p2_mul", k_fmul<FieldP2>, occ, 1, ITERS, d_cyc, d_out, false);
            run("p2_sqr", k_fsqr<FieldP2>, occ, 1, ITERS, d_cyc, d_out, false);
            run("n2_mul_generic", k_fmul<FieldN2>, occ, 1, ITERS, d_cyc, d_out, false);
            run("n2_sqr_generic", k_fsqr<FieldN2>, occ, 1, ITERS, d_cyc, d_out, false);
        }
        run("fk1_mul_chain1", k_mul<1>, occ, 1, ITERS, d_cyc, d_out, false);
        run("fk1_mul_chain2", k_mul<2>, occ, 2, ITERS, d_cyc, d_out, false);
        run("fk1_sqr_chain1", k_sqr<1>, occ, 1, ITERS, d_cyc, d_out, false);
        run("fk1_sqr_chain2", k_sqr<2>, occ, 2, ITERS, d_cyc, d_out, false);
        run("f26_mul_chain1", k_f26mul<1>, occ, 1, ITERS, d_cyc, d_out, false);
        run("f26_mul_chain2", k_f26mul<2>, occ, 2, ITERS, d_cyc, d_out, false);
        run("f26_sqr_chain1", k_f26sqr<1>, occ, 1, ITERS, d_cyc, d_out, false);
        run("f26_sqr_chain2", k_f26sqr<2>, occ, 2, ITERS, d_cyc, d_out, false);
        run("k1_dbl", k_dbl, occ, 1, ITERS / 8, d_cyc, d_out, false);
        run("f26_dbl", k_f26dbl, occ, 1, ITERS / 8, d_cyc, d_out, false);
        run("k1_madd", k_madd, occ, 1, ITERS / 8, d_cyc, d_out, false);
        run("f26_madd", k_f26madd, occ, 1, ITERS / 8, d_cyc, d_out, occ == 4);
    }
    printf("}\n");
    return 0;
}
