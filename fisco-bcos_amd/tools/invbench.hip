// invbench.hip -- cycles of the safegcd inversion (modinv.h) on a lone wave: the plain loop against the
// software-pipelined one (the (d, e) update beside the next batch's divsteps), plus the parts of one
// batch (30 divsteps, the (f, g) and (d, e) updates), and agreement of the two variants on random
// inputs mod p (secp256k1) and mod n.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../csrc/modinv.h"
using namespace bcosgpu;

__global__ void inv_kernel(const fe* in, fe* out_a, fe* out_b, int which_mod, uint64_t* cyc) {
    const ModInfo30& mi = which_mod ? kMod30N1 : kMod30K1P;
    const fe x = in[threadIdx.x];
    fe a, b;
    __syncthreads();
    uint64_t t0 = clock64();
    modinv_safegcd(a, x, mi);
    uint64_t t1 = clock64();
    fe x2;
    fe_copy(x2, x);
    x2.v[0] ^= a.v[0] & 0u;  // keep the order of the two timed regions
    uint64_t t2 = clock64();
    modinv_safegcd_pipe(b, x2, mi);
    uint64_t t3 = clock64();
    out_a[threadIdx.x] = a;
    out_b[threadIdx.x] = b;
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t3 - t2;
    }
}

__global__ void parts_kernel(const fe* in, uint64_t* cyc, int32_t* sink) {
    S30 d, e, f, g;
    fe_to_s30(f, in[threadIdx.x]);
    fe_to_s30(g, in[(threadIdx.x + 1) & 63]);
    fe_to_s30(d, in[(threadIdx.x + 2) & 63]);
    fe_to_s30(e, in[(threadIdx.x + 3) & 63]);
    f.v[0] |= 1;
    int32_t t[4] = {1, 0, 0, 1}, zeta = -1;
    uint64_t t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 20; ++i) zeta = divsteps_30(zeta, static_cast<uint32_t>(f.v[0]) + i, static_cast<uint32_t>(g.v[0]) ^ zeta, t);
    uint64_t t1 = clock64();
#pragma unroll 1
    for (int i = 0; i < 20; ++i) update_fg_30(f, g, t);
    uint64_t t2 = clock64();
#pragma unroll 1
    for (int i = 0; i < 20; ++i) update_de_30(d, e, t, kMod30K1P);
    uint64_t t3 = clock64();
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / 20;
        cyc[1] = (t2 - t1) / 20;
        cyc[2] = (t3 - t2) / 20;
    }
    int32_t s = zeta;
    for (int i = 0; i < 9; ++i) s ^= d.v[i] ^ e.v[i] ^ f.v[i] ^ g.v[i];
    sink[threadIdx.x] = s;
}

// the variable-time inversion (modinv_safegcd_var), one timed region per launch: mode 0 per-lane inputs
// (the wave runs its slowest lane), 1 one value in every lane, 2 that value made uniform (readfirstlane:
// the compiler may keep it in SGPRs); mode 3 the pipelined constant-time loop on one value in every lane
template <int U>
__global__ void var_kernel(const fe* in, fe* out, int which_mod, int mode, uint64_t* cyc) {
    const ModInfo30& mi = which_mod ? kMod30N1 : kMod30K1P;
    fe x = in[mode == 0 ? threadIdx.x : 0];
    if (mode == 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x.v[k] = __builtin_amdgcn_readfirstlane(x.v[k]);
    }
    fe a;
    __syncthreads();
    const uint64_t t0 = clock64();
    if (mode == 3) modinv_safegcd_pipe(a, x, mi);
    else modinv_safegcd_var<U>(a, x, mi);
    out[threadIdx.x] = a;
    __syncthreads();
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    std::vector<fe> x(64);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& v : x)
        for (int i = 0; i < 8; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            v.v[i] = static_cast<uint32_t>(s);
        }
    for (auto& v : x) v.v[7] &= 0x7fffffffu;  // < both moduli
    fe *dx, *da, *db;
    uint64_t* dc;
    int32_t* dk;
    if (hipMalloc(&dx, 64 * sizeof(fe)) != hipSuccess) return 77;
    (void)hipMalloc(&da, 64 * sizeof(fe)); (void)hipMalloc(&db, 64 * sizeof(fe));
    (void)hipMalloc(&dc, 64); (void)hipMalloc(&dk, 256);
    (void)hipMemcpy(dx, x.data(), 64 * sizeof(fe), hipMemcpyHostToDevice);
    int bad = 0;
    uint64_t c[4][2];
    for (int m = 0; m < 2; ++m) {
        for (int rep = 0; rep < 2; ++rep) {  // second run timed warm
            hipLaunchKernelGGL(inv_kernel, dim3(1), dim3(64), 0, 0, dx, da, db, m, dc);
            (void)hipMemcpy(c[2 * m + rep], dc, 16, hipMemcpyDeviceToHost);
        }
        std::vector<fe> a(64), b(64);
        (void)hipMemcpy(a.data(), da, 64 * sizeof(fe), hipMemcpyDeviceToHost);
        (void)hipMemcpy(b.data(), db, 64 * sizeof(fe), hipMemcpyDeviceToHost);
        for (int i = 0; i < 64; ++i)
            for (int k = 0; k < 8; ++k) bad += a[i].v[k] != b[i].v[k];
    }
    // the variable-time loop at four unroll depths: each lane's result against the constant-time one;
    // cycles [mod][unroll][mode]
    fe* dv;
    (void)hipMalloc(&dv, 64 * sizeof(fe));
    uint64_t cv[2][4][4];
    for (int m = 0; m < 2; ++m) {
        hipLaunchKernelGGL(inv_kernel, dim3(1), dim3(64), 0, 0, dx, da, db, m, dc);
        std::vector<fe> a(64), v(64);
        (void)hipMemcpy(a.data(), da, 64 * sizeof(fe), hipMemcpyDeviceToHost);
        for (int uu = 0; uu < 4; ++uu)
            for (int mode = 0; mode < 4; ++mode) {
                for (int rep = 0; rep < 2; ++rep) {
                    if (uu == 0) hipLaunchKernelGGL(var_kernel<2>, dim3(1), dim3(64), 0, 0, dx, dv, m, mode, dc);
                    else if (uu == 1) hipLaunchKernelGGL(var_kernel<3>, dim3(1), dim3(64), 0, 0, dx, dv, m, mode, dc);
                    else if (uu == 2) hipLaunchKernelGGL(var_kernel<4>, dim3(1), dim3(64), 0, 0, dx, dv, m, mode, dc);
                    else hipLaunchKernelGGL(var_kernel<6>, dim3(1), dim3(64), 0, 0, dx, dv, m, mode, dc);
                    (void)hipMemcpy(&cv[m][uu][mode], dc, 8, hipMemcpyDeviceToHost);
                }
                (void)hipMemcpy(v.data(), dv, 64 * sizeof(fe), hipMemcpyDeviceToHost);
                for (int i = 0; i < 64; ++i)
                    for (int k = 0; k < 8; ++k) bad += v[i].v[k] != a[mode == 0 ? i : 0].v[k];
            }
    }
    printf("{\"var_mismatched_words\": %d, \"cycles[mod p, n][unroll 2, 3, 4, 6][lanes, same, uniform, const_pipe_same]\": [",
           bad);
    for (int m = 0; m < 2; ++m)
        for (int uu = 0; uu < 4; ++uu)
            printf("%s[%llu, %llu, %llu, %llu]", (m | uu) ? ", " : "", (unsigned long long)cv[m][uu][0],
                   (unsigned long long)cv[m][uu][1], (unsigned long long)cv[m][uu][2], (unsigned long long)cv[m][uu][3]);
    printf("]}\n");
    uint64_t p[3];
    hipLaunchKernelGGL(parts_kernel, dim3(1), dim3(64), 0, 0, dx, dc, dk);
    (void)hipMemcpy(p, dc, 24, hipMemcpyDeviceToHost);
    printf("{\"mismatched_words\": %d, \"inv_p_cycles\": %llu, \"inv_p_pipe_cycles\": %llu, \"inv_n_cycles\": %llu, "
           "\"inv_n_pipe_cycles\": %llu, \"divsteps30_cycles\": %llu, \"update_fg_cycles\": %llu, \"update_de_cycles\": %llu}\n",
           bad, (unsigned long long)c[1][0], (unsigned long long)c[1][1], (unsigned long long)c[3][0],
           (unsigned long long)c[3][1], (unsigned long long)p[0], (unsigned long long)p[1], (unsigned long long)p[2]);
    return bad ? 1 : 0;
}
