// triobench.hip -- the lane-trio point operations (csrc/ec26_trio.h) against the one-lane CurveK1x
// ones: the same windows (4 doublings + 1 mixed addition) from the same random inputs, results
// compared on the host, and s_memtime cycles per window of a lone wave per SIMD for both.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
__device__ unsigned int g_dump[64][8][10];
#define TRIO_DUMP(slot, a)                                                                  \
    do {                                                                                    \
        if (blockIdx.x == 0 && threadIdx.x < 64) {                                          \
            fe26 _t = (a);                                                                  \
            fe26_normalize(_t);                                                             \
            for (int _i = 0; _i < 10; ++_i) g_dump[threadIdx.x][slot][_i] = _t.v[_i];       \
        }                                                                                   \
    } while (0)
#include "../csrc/ec26_trio.h"

using namespace bcosgpu;

__device__ __forceinline__ void load_fe26(fe26& a, const uint32_t* p) {
    uint32_t w[8];
    for (int i = 0; i < 8; ++i) w[i] = p[i];
    w[7] &= 0x7fffffffu;
    fe26_from_words(a, w);
}

// mode 0: trio, mode 1: one lane per point (every lane of a trio computes its point)
__global__ __launch_bounds__(256, 1) void trio_bench(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     unsigned long long* __restrict__ cyc, int iters, int mode, int ops) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = lane >> 4, pos = lane & 15, t = pos / 3;
    const int tt = t < 5 ? t : 4;
    const int pid = (blockIdx.x * 4 + wave) * 20 + row * 5 + tt;
    const uint32_t* p = in + pid * 40;
    Jac26 J;
    Aff26 Q;
    load_fe26(J.X, p);
    load_fe26(J.Y, p + 8);
    load_fe26(J.Z, p + 16);
    load_fe26(Q.x, p + 24);
    load_fe26(Q.y, p + 32);
    J.inf = false;
    const TrioLane T(lane);
    unsigned long long t0 = 0, t1 = 0;
    if (mode == 0) {
        TrioPt P;
        trio::sel(P.S1, T.r0, J.X, J.Y);
        fe26_copy(P.Xs, J.X);
        fe26_copy(P.Zs, J.Z);
        P.inf = false;
        t0 = clock64();
#pragma unroll 1
        for (int it = 0; it < iters; ++it) {
            if (ops & 1) {
                trio_dbl(P, T);
                trio_dbl(P, T);
                trio_dbl(P, T);
                trio_dbl(P, T);
            }
            if (ops & 2) trio_madd(P, P, Q, T);
            if (ops & 4) {  // the kernel's window: 3 doublings, the Z^2-carrying one, the 4-level addition
                fe26 zz;
                trio_dbl(P, T);
                trio_dbl(P, T);
                trio_dbl(P, T);
                trio_dbl_zz(P, zz, T);
                trio_madd_zz(P, P, zz, Q, T);
            }
        }
        t1 = clock64();
        trio_to_jac(J, P, T);
    } else {
        t0 = clock64();
#pragma unroll 1
        for (int it = 0; it < iters; ++it) {
            if (ops & 1) {
                CurveK1x::dbl(J, J);
                CurveK1x::dbl(J, J);
                CurveK1x::dbl(J, J);
                CurveK1x::dbl(J, J);
            }
            if (ops & 6) {
                if (ops & 4) {
                    CurveK1x::dbl(J, J);
                    CurveK1x::dbl(J, J);
                    CurveK1x::dbl(J, J);
                    CurveK1x::dbl(J, J);
                }
                Jac26 R;
                CurveK1x::madd(R, J, Q);
                J = R;
            }
        }
        t1 = clock64();
    }
    fe26_normalize(J.X);
    fe26_normalize(J.Y);
    fe26_normalize(J.Z);
    if (T.r0 && t < 5) {
        uint32_t* o = out + pid * 32;
        fe26_to_words(o, J.X);
        fe26_to_words(o + 8, J.Y);
        fe26_to_words(o + 16, J.Z);
        o[24] = J.inf ? 1u : 0u;
    }
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

__global__ void dpp_probe(uint32_t* out) {
    const uint32_t l = threadIdx.x;
    out[l] = trio::dpp<trio::kL1>(l + 100);
    out[64 + l] = trio::dpp<trio::kR1>(l + 100);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 64, iters = argc > 2 ? atoi(argv[2]) : 32;
    const int ops = argc > 3 ? atoi(argv[3]) : 3;
    const int npts = blocks * 4 * 20;
    std::vector<uint32_t> in(npts * 40), o0(npts * 32), o1(npts * 32);
    uint32_t x = 987654321u;
    for (auto& w : in) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; w = x; }
    uint32_t *din, *dout;
    unsigned long long* dcyc;
    if (hipMalloc(&din, in.size() * 4) != hipSuccess) { printf("no device\n"); return 77; }
    hipMalloc(&dout, o0.size() * 4);
    hipMalloc(&dcyc, blocks * 4 * 8);
    hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice);
    std::vector<unsigned long long> c(blocks * 4);
    double cw[2] = {0, 0};
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(trio_bench, dim3(blocks), dim3(256), 0, 0, din, dout, dcyc, iters, mode, ops);
            hipDeviceSynchronize();
        }
        hipMemcpy(mode ? o1.data() : o0.data(), dout, o0.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
        unsigned long long s = 0;
        for (auto v : c) s += v;
        cw[mode] = double(s) / c.size() / iters;
    }
    {
        hipLaunchKernelGGL(dpp_probe, dim3(1), dim3(64), 0, 0, dout);
        std::vector<uint32_t> pr(128);
        hipMemcpy(pr.data(), dout, 512, hipMemcpyDeviceToHost);
        printf("dpp L1 lanes 0..17:");
        for (int i = 0; i < 18; ++i) printf(" %u", pr[i]);
        printf("\ndpp R1 lanes 0..17:");
        for (int i = 0; i < 18; ++i) printf(" %u", pr[64 + i]);
        printf("\n");
    }
    if (ops == 2 && iters == 1) {  // intermediate values of trio 0 against a host recomputation
        static unsigned int dump[64][8][10];
        hipMemcpyFromSymbol(dump, HIP_SYMBOL(g_dump), sizeof(dump));
        const uint32_t* p = in.data();
        auto ld = [](fe26& a, const uint32_t* q) { uint32_t w[8]; for (int i = 0; i < 8; ++i) w[i] = q[i]; w[7] &= 0x7fffffffu; fe26_from_words(a, w); };
        fe26 X, Y, Z, x2, y2, Z1Z1, yZ, U2, S2, H, rr, HH, R2, ZH, I, J, V, X3, t, W, a5, b5, Y3;
        ld(X, p); ld(Y, p + 8); ld(Z, p + 16); ld(x2, p + 24); ld(y2, p + 32);
        fe26_sqr(Z1Z1, Z); fe26_mul(yZ, y2, Z); fe26_mul(U2, x2, Z1Z1); fe26_mul(S2, yZ, Z1Z1);
        fe26_sub<11>(H, U2, X); fe26_sub<11>(rr, S2, Y); fe26_sqr(HH, H); fe26_sqr(R2, rr); fe26_mul(ZH, Z, H);
        fe26_mul_int<4>(I, HH); fe26_mul(J, H, I); fe26_mul(V, X, I);
        fe26 R4; fe26_mul_int<4>(R4, R2); fe26_sub<2>(X3, R4, J); fe26_mul_int<2>(t, V); fe26_sub<3>(X3, X3, t);
        fe26_sub<10>(W, V, X3); fe26_mul(a5, rr, W); fe26_mul(b5, Y, J); fe26_sub<2>(Y3, a5, b5); fe26_mul_int<2>(Y3, Y3);
        const fe26* want[8][3] = {{&Z1Z1, &yZ, &Z1Z1}, {&U2, &S2, &U2}, {&H, &rr, &H}, {&HH, &R2, &ZH},
                                  {&J, nullptr, &V}, {&a5, &b5, nullptr}, {&X3, nullptr, nullptr}, {&Y3, nullptr, nullptr}};
        for (int sl = 0; sl < 8; ++sl)
            for (int ln = 0; ln < 3; ++ln) {
                if (!want[sl][ln]) continue;
                fe26 e = *want[sl][ln];
                fe26_normalize(e);
                printf("slot %d lane %d: %s\n", sl, ln, memcmp(e.v, dump[ln][sl], 40) ? "DIFF" : "ok");
            }
    }
    int bad = 0;
    for (int i = 0; i < npts; ++i)
        if (memcmp(&o0[i * 32], &o1[i * 32], 25 * 4)) ++bad;
    printf("{\"points\": %d, \"mismatch\": %d, \"cycles_per_window_trio\": %.0f, \"cycles_per_window_one_lane\": %.0f, "
           "\"ops\": %d}\n", npts, bad, cw[0], cw[1], ops);
    return bad ? 1 : 0;
}
