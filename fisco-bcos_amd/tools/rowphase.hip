// rowphase.hip -- phase timestamps (s_memtime cycles) of the row kernel's workgroup 0 (ecc_row.hip,
// recover_row_kernel<SigIO>) on a batch of 16 random signatures, to see where a recovery's latency goes.
#define BCOSGPU_ROW_TIMING 1
#include "../csrc/ecc_tables.hip"
#include "../csrc/ecc_row.hip"
#include <cstdio>
#include <vector>

int main() {
    using namespace bcosgpu;
    if (ecc_init_tables(0, 0)) {
        printf("no device\n");
        return 77;
    }
    const uint64_t n = 16;
    std::vector<uint8_t> h(32 * n), sig(65 * n);
    uint32_t x = 12345;
    for (auto& b : h) b = (x = x * 1103515245u + 12345u) >> 24;
    for (auto& b : sig) b = (x = x * 1103515245u + 12345u) >> 24;
    for (uint64_t i = 0; i < n; ++i) {
        sig[65 * i] &= 0x7f;  // r < n
        sig[65 * i + 32] &= 0x7f;
        sig[65 * i + 64] = i & 1;
    }
    uint8_t *dh, *ds, *dpub, *dad, *dok;
    hipMalloc(&dh, h.size());
    hipMalloc(&ds, sig.size());
    hipMalloc(&dpub, 64 * n);
    hipMalloc(&dad, 20 * n);
    hipMalloc(&dok, n);
    hipMemcpy(dh, h.data(), h.size(), hipMemcpyHostToDevice);
    hipMemcpy(ds, sig.data(), sig.size(), hipMemcpyHostToDevice);
    const SigIO io{dh, ds, 65u, 65u, dpub, dad, dok};
    for (int rep = 0; rep < 5; ++rep) launch_recover_row(io, n, 0);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    uint64_t t[4][8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_row_t), sizeof(t));
    printf("{\"cycles_since_start\": {");
    for (int w = 0; w < 4; ++w)
        printf("%s\"wave%d\": [%llu, %llu, %llu]", w ? ", " : "", w, (unsigned long long)(t[w][1] - t[w][0]),
               (unsigned long long)(t[w][2] - t[w][0]), (unsigned long long)(t[w][3] - t[w][0]));
    printf("}, \"comb_done\": [%llu, %llu, %llu, %llu], \"wave0_inversion\": [%llu, %llu], \"probes\": \"phase-A work "
           "done, chain done, end of kernel; comb partial done per wave; wave 0: before / after the affine inversion\"}\n",
           (unsigned long long)(t[0][6] - t[0][0]), (unsigned long long)(t[1][6] - t[1][0]),
           (unsigned long long)(t[2][6] - t[2][0]), (unsigned long long)(t[3][6] - t[3][0]),
           (unsigned long long)(t[0][4] - t[0][0]), (unsigned long long)(t[0][5] - t[0][0]));
    return 0;
}
