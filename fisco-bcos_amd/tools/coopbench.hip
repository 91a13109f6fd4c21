// coopbench.hip -- phase timestamps (s_memtime cycles) of tx_verify_coop_kernel's (argv[1] = 26:
// tx_verify_coop26_kernel's, trio: tx_verify_trio26_kernel's) workgroup 0 on a
// 10k-tx batch of random inputs (the schedule is input-independent), to see where C2's latency goes.
#define BCOSGPU_COOP_TIMING 1
#include "../csrc/ecc_tables.hip"
#include "../csrc/ecc_coop.hip"
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    using namespace bcosgpu;
    const bool f26 = argc > 1 && argv[1][0] == '2';  // "26": tx_verify_coop26_kernel
    const bool trio = argc > 1 && argv[1][0] == 't';  // "trio": tx_verify_trio26_kernel (16-bit comb)
    if (ecc_init_tables(0, trio ? 0 : 1)) { printf("no device\n"); return 77; }
    const uint64_t n = 10000;
    std::vector<uint8_t> pre(n * 151), sig(n * 65);
    std::vector<uint64_t> po(n + 1), so(n + 1);
    uint32_t x = 12345;
    for (auto& b : pre) b = (x = x * 1103515245u + 12345u) >> 24;
    for (auto& b : sig) b = (x = x * 1103515245u + 12345u) >> 24;
    for (uint64_t i = 0; i <= n; ++i) { po[i] = 151 * i; so[i] = 65 * i; }
    for (uint64_t i = 0; i < n; ++i) sig[65 * i + 64] = 0;
    uint8_t *dp, *ds, *dh, *dsn, *dst;
    uint64_t *dpo, *dso;
    hipMalloc(&dp, pre.size()); hipMalloc(&ds, sig.size()); hipMalloc(&dpo, 8 * (n + 1)); hipMalloc(&dso, 8 * (n + 1));
    hipMalloc(&dh, 32 * n); hipMalloc(&dsn, 20 * n); hipMalloc(&dst, n);
    hipMemcpy(dp, pre.data(), pre.size(), hipMemcpyHostToDevice);
    hipMemcpy(ds, sig.data(), sig.size(), hipMemcpyHostToDevice);
    hipMemcpy(dpo, po.data(), 8 * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(dso, so.data(), 8 * (n + 1), hipMemcpyHostToDevice);
    const uint32_t *k1, *sm2;
    tables8(&k1, &sm2);
    const TxIO io{dp, dpo, ds, dso, dh, dsn, dst};
    for (int rep = 0; rep < 3; ++rep) {
        if (trio) {
            const uint32_t *w1, *w2;
            int bits = 8;
            tables(&w1, &w2, &bits);
            hipLaunchKernelGGL(tx_verify_trio26_kernel<TxIO>, dim3((n + 39) / 40), dim3(256), 0, 0, io, n, w1, bits);
        } else if (f26)
            hipLaunchKernelGGL(tx_verify_coop26_kernel<TxIO>, dim3((n + 63) / 64), dim3(256), 0, 0, io, n, k1);
        else
            hipLaunchKernelGGL(tx_verify_coop_kernel, dim3((n + 63) / 64), dim3(256), 0, 0, dp, dpo, ds, dso, n, k1, dh,
                               dsn, dst);
        hipDeviceSynchronize();
    }
    uint64_t t[4][8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_coop_t), sizeof(t));
    printf("{\"cycles_since_start\": {");
    for (int w = 0; w < 4; ++w)
        printf("%s\"wave%d\": [%llu, %llu, %llu]", w ? ", " : "", w, (unsigned long long)(t[w][1] - t[w][0]),
               (unsigned long long)(t[w][2] - t[w][0]), (unsigned long long)(t[w][3] - t[w][0]));
    printf("}, \"probes6_7\": [");
    for (int w = 0; w < 4; ++w)
        printf("%s[%llu, %llu]", w ? ", " : "", (unsigned long long)(t[w][6] - t[w][0]), (unsigned long long)(t[w][7] - t[w][0]));
    uint64_t dt[4][8];
    hipMemcpyFromSymbol(dt, HIP_SYMBOL(g_dbl_t), sizeof(dt));
    printf("], \"dbl\": [");
    for (int w = 0; w < 4; ++w)
        printf("%s[%llu, %llu, %llu, %llu, %llu, %llu, %llu]", w ? ", " : "", (unsigned long long)(dt[w][1] - dt[w][0]),
               (unsigned long long)(dt[w][2] - dt[w][0]), (unsigned long long)(dt[w][3] - dt[w][0]),
               (unsigned long long)(dt[w][4] - dt[w][0]), (unsigned long long)(dt[w][5] - dt[w][0]),
               (unsigned long long)(dt[w][6] - dt[w][0]), (unsigned long long)(dt[w][7] - dt[w][0]));
    printf("], \"wave0_phase_d\": [%llu, %llu], \"probes\": \"end of phase A work, end of phase C loop, end of kernel; wave 0: before / after the affine inversion\"}\n",
           (unsigned long long)(t[0][4] - t[0][0]), (unsigned long long)(t[0][5] - t[0][0]));
    return 0;
}
