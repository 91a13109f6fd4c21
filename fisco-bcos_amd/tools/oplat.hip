// oplat.hip -- cycles per instruction of one lone wave (one wave per SIMD) for the VALU operations the
// fe26 / trio code is made of: one dependency chain (latency) and eight independent chains (issue),
// s_memtime around 512 iterations.  Prints JSON {op: [chain1_cycles, chain8_cycles_per_instr]}.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 512

#define OPK(NAME, T, ASM)                                                                  \
    template <int CH>                                                                      \
    __global__ __launch_bounds__(256) void NAME(uint64_t* cyc, uint32_t seed) {            \
        T x[CH];                                                                           \
        const uint32_t c = seed | 1u;                                                      \
        for (int k = 0; k < CH; ++k) x[k] = static_cast<T>(threadIdx.x * 7919u + k + seed); \
        const uint64_t t0 = clock64();                                                     \
        _Pragma("unroll 16") for (int it = 0; it < ITERS; ++it) {                          \
            _Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(ASM : "+v"(x[k]) : "v"(c)); \
        }                                                                                  \
        const uint64_t t1 = clock64();                                                     \
        T r = 0;                                                                           \
        for (int k = 0; k < CH; ++k) r ^= x[k];                                            \
        if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;                         \
        if (r == static_cast<T>(0x12345678u)) cyc[1] = static_cast<uint64_t>(r);           \
    }

OPK(k_and, uint32_t, "v_and_b32 %0, %0, %1")
OPK(k_add, uint32_t, "v_add_u32 %0, %0, %1")
OPK(k_cndmask, uint32_t, "v_cndmask_b32 %0, %0, %1, vcc")
OPK(k_dpp, uint32_t, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1")
OPK(k_dpp_nonop, uint32_t, "v_add_u32 %0, %0, %1\n\tv_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
OPK(k_lshr64, uint64_t, "v_lshrrev_b64 %0, 26, %0")
OPK(k_lshladd64, uint64_t, "v_lshl_add_u64 %0, %0, 2, %0")
OPK(k_alignbit, uint32_t, "v_alignbit_b32 %0, %0, %1, 26")

template <int CH>
__global__ __launch_bounds__(256) void k_mad64(uint64_t* cyc, uint32_t seed) {
    uint64_t x[CH];
    const uint32_t c = seed | 1u;
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            uint64_t cc;
            const uint32_t lo = static_cast<uint32_t>(x[k]);
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x[k]), "=s"(cc) : "v"(lo), "v"(c));
        }
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}


// eight chains whose carry-outs go to eight distinct SGPR pairs ("+s": each stays allocated)
template <int CH>
__global__ __launch_bounds__(256) void k_mad64_sj(uint64_t* cyc, uint32_t seed) {
    uint64_t x[CH], cc[CH];
    const uint32_t c = seed | 1u;
    for (int k = 0; k < CH; ++k) {
        x[k] = threadIdx.x * 7919u + k + seed;
        cc[k] = k;
    }
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const uint32_t lo = static_cast<uint32_t>(x[k]);
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x[k]), "+s"(cc[k]) : "v"(lo), "v"(c));
        }
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k] ^ cc[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}
// eight chains, carry-outs to VCC (one pair, as the fe26 blocks' junk)
template <int CH>
__global__ __launch_bounds__(256) void k_mad64_vcc(uint64_t* cyc, uint32_t seed) {
    uint64_t x[CH];
    const uint32_t c = seed | 1u;
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const uint32_t lo = static_cast<uint32_t>(x[k]);
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[k]) : "v"(lo), "v"(c) : "vcc");
        }
    }
    const uint64_t t1 = clock64();
    uint64_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}
// eight chains of v_mad_u32_u24 (no SGPR output) and of v_mul_hi_u32 (VOP3, no SGPR output)
OPK(k_mad24, uint32_t, "v_mad_u32_u24 %0, %0, %1, %0")
OPK(k_mulhi, uint32_t, "v_mul_hi_u32 %0, %0, %1")
OPK(k_mullo, uint32_t, "v_mul_lo_u32 %0, %0, %1")


// v_cndmask with the mask in an SGPR pair (e64) set once by the compiler, and in VCC set by s_mov
template <int CH>
__global__ __launch_bounds__(256) void k_cnd_sgpr(uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
    const uint32_t c = seed | 1u;
    const uint64_t m = __builtin_amdgcn_ballot_w64((threadIdx.x & 3) == 1);
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CH; ++k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[k]) : "v"(c), "s"(m));
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}
template <int CH>
__global__ __launch_bounds__(256) void k_cnd_vccset(uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
    const uint32_t c = seed | 1u;
    const uint64_t m = __builtin_amdgcn_ballot_w64((threadIdx.x & 3) == 1);
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
        asm volatile("s_mov_b64 vcc, %0\n\ts_nop 1" : : "s"(m) : "vcc");
#pragma unroll
        for (int k = 0; k < CH; ++k) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(c) : "vcc");
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}
// c ? a : b compiled by the compiler (what fe26 sel / cmov become)
template <int CH>
__global__ __launch_bounds__(256) void k_sel_cc(uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
    const uint32_t c = seed | 1u;
    const bool p = (threadIdx.x % 3) == 1;
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 7919u + k + seed;
    const uint64_t t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            x[k] = p ? x[k] + c : x[k] ^ c;
            asm volatile("" : "+v"(x[k]));
        }
    }
    const uint64_t t1 = clock64();
    uint32_t r = 0;
    for (int k = 0; k < CH; ++k) r ^= x[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (r == 0x12345678u) cyc[1] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);
static double per_instr(kfn f, uint64_t* d, int ch, int ninstr) {
    hipLaunchKernelGGL(f, dim3(1), dim3(256), 0, 0, d, 3u);  // 4 waves, one per SIMD
    hipLaunchKernelGGL(f, dim3(1), dim3(256), 0, 0, d, 3u);
    uint64_t c = 0;
    (void)hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
    return static_cast<double>(c) / (static_cast<double>(ITERS) * ch * ninstr);
}

int main() {
    uint64_t* d;
    if (hipMalloc(&d, 64) != hipSuccess) return 77;
    struct { const char* name; kfn f1, f8; int n; } ks[] = {
        {"v_and_b32", k_and<1>, k_and<8>, 1}, {"v_add_u32", k_add<1>, k_add<8>, 1},
        {"v_cndmask_b32", k_cndmask<1>, k_cndmask<8>, 1}, {"v_mov_b32_dpp+s_nop1", k_dpp<1>, k_dpp<8>, 1},
        {"v_add+v_mov_b32_dpp", k_dpp_nonop<1>, k_dpp_nonop<8>, 2}, {"v_lshrrev_b64", k_lshr64<1>, k_lshr64<8>, 1},
        {"v_lshl_add_u64", k_lshladd64<1>, k_lshladd64<8>, 1}, {"v_alignbit_b32", k_alignbit<1>, k_alignbit<8>, 1},
        {"v_mad_u64_u32", k_mad64<1>, k_mad64<8>, 1}, {"v_mad_u64_u32 distinct sgpr", k_mad64_sj<1>, k_mad64_sj<8>, 1},
        {"v_mad_u64_u32 vcc", k_mad64_vcc<1>, k_mad64_vcc<8>, 1}, {"v_mad_u32_u24", k_mad24<1>, k_mad24<8>, 1},
        {"v_mul_hi_u32", k_mulhi<1>, k_mulhi<8>, 1}, {"v_mul_lo_u32", k_mullo<1>, k_mullo<8>, 1},
        {"v_cndmask_b32_e64 sgpr mask", k_cnd_sgpr<1>, k_cnd_sgpr<8>, 1},
        {"v_cndmask_b32 vcc (s_mov)", k_cnd_vccset<1>, k_cnd_vccset<8>, 1},
        {"compiler select (add|xor, cndmask)", k_sel_cc<1>, k_sel_cc<8>, 3}};
    printf("{\"note\": \"cycles per instruction, lone wave per SIMD: [one dependency chain, eight chains]\"");
    for (auto& k : ks) printf(", \"%s\": [%.2f, %.2f]", k.name, per_instr(k.f1, d, 1, k.n), per_instr(k.f8, d, 8, k.n));
    printf("}\n");
    return 0;
}
