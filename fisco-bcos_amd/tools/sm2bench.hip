// sm2bench.hip -- phase timestamps (s_memtime cycles) of tx_verify_sm2_trio26_kernel's workgroup 0 on a
// 10k-tx batch of random inputs (the schedule is input-independent), to see where c2sm2's latency goes.
//   sm2bench [REPS [SYNTH_DIR | - [SPLIT]]]   (SPLIT in 0, 40, 42, 44, 46, 48)
#define BCOSGPU_SM2_TIMING 1
#include "../csrc/ecc_tables.hip"
#ifdef SM2BENCH_PAIR_SRC  // A/B builds: another revision of ecc_pair.hip, whose kernel takes no 'affine' flag
#include SM2BENCH_PAIR_SRC
#define SM2_AFFINE_ARG
#else
#include "../csrc/ecc_pair.hip"
#define SM2_AFFINE_ARG , 1, ctab, cbits
#define SM2_SPLIT_ARG(S) , S
#endif
#ifndef SM2_SPLIT_ARG
#define SM2_SPLIT_ARG(S)
#endif
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 4;
    // low Booth windows on waves 2 and 3 (sm2_low_chain): argv[3], else the library's default
    const int split = argc > 3 ? atoi(argv[3]) : bcosgpu::kSm2TrioSplit;
    using namespace bcosgpu;
    if (ecc_init_tables(0, 0)) { printf("no device\n"); return 77; }
    const uint64_t n = 10000;
    uint64_t plen = 151;
    std::vector<uint8_t> pre(n * plen), sig(n * 128);
    uint32_t x = 12345;
    for (auto& b : pre) b = (x = x * 1103515245u + 12345u) >> 24;
    for (auto& b : sig) b = (x = x * 1103515245u + 12345u) >> 24;
    if (argc > 2 && std::string(argv[2]) != "-") {  // the bench's batch (tools/dump_synth.py <dir>): valid signatures
        const std::string d = argv[2];
        FILE* f = fopen((d + "/pre.bin").c_str(), "rb");
        FILE* g = fopen((d + "/sig.bin").c_str(), "rb");
        if (!f || !g) { printf("no synth files\n"); return 1; }
        fseek(f, 0, SEEK_END);
        plen = static_cast<uint64_t>(ftell(f)) / n;
        fseek(f, 0, SEEK_SET);
        pre.resize(n * plen);
        if (fread(pre.data(), 1, pre.size(), f) != pre.size() || fread(sig.data(), 1, sig.size(), g) != sig.size()) {
            printf("short synth files\n");
            return 1;
        }
        fclose(f);
        fclose(g);
    }
    std::vector<uint64_t> po(n + 1), so(n + 1);
    for (uint64_t i = 0; i <= n; ++i) { po[i] = plen * i; so[i] = 128 * i; }
    uint8_t *dp, *ds, *dh, *dsn, *dst;
    uint64_t *dpo, *dso;
    hipMalloc(&dp, pre.size()); hipMalloc(&ds, sig.size()); hipMalloc(&dpo, 8 * (n + 1)); hipMalloc(&dso, 8 * (n + 1));
    hipMalloc(&dh, 32 * n); hipMalloc(&dsn, 20 * n); hipMalloc(&dst, n);
    hipMemcpy(dp, pre.data(), pre.size(), hipMemcpyHostToDevice);
    hipMemcpy(ds, sig.data(), sig.size(), hipMemcpyHostToDevice);
    hipMemcpy(dpo, po.data(), 8 * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(dso, so.data(), 8 * (n + 1), hipMemcpyHostToDevice);
    const uint32_t* t26;
    if (tables8_sm2_26(&t26)) { printf("no table\n"); return 1; }
    const uint32_t* ctab = t26;  // s G's comb: the 16-bit R'-domain table when present (as the library)
    int cbits = 8;
    if (tables_sm2_26(&ctab, &cbits)) { ctab = t26; cbits = 8; }
    const TxIO io{dp, dpo, ds, dso, dh, dsn, dst};
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0;
    // reps back-to-back launches (the clock settles under load); the mean over the last half is reported
    for (int rep = 0; rep < reps; ++rep) {
        if (rep == reps / 2) hipEventRecord(e0);
        switch (split) {  // the split is a template parameter of the kernel: the instantiations swept here
#define SM2_CASE(S) \
    case S: hipLaunchKernelGGL((tx_verify_sm2_trio26_kernel<TxIO SM2_SPLIT_ARG(S)>), dim3((n + 39) / 40), dim3(256), 0, 0, io, n, t26 SM2_AFFINE_ARG); break;
            SM2_CASE(0) SM2_CASE(40) SM2_CASE(42) SM2_CASE(44) SM2_CASE(46) SM2_CASE(48)
#undef SM2_CASE
            default: printf("split %d not instantiated\n", split); return 1;
        }
        if (rep % 64 == 63) hipDeviceSynchronize();
    }
    hipEventRecord(e1);
    hipDeviceSynchronize();
    hipEventElapsedTime(&ms, e0, e1);
    ms /= static_cast<float>(reps - reps / 2);
    uint64_t t[4][8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_sm2_t), sizeof(t));
    printf("{\"split\": %d, \"comb_bits\": %d, \"kernel_ms\": %.4f, \"cycles_since_start\": {", split, cbits, ms);
    for (int w = 0; w < 4; ++w)
        printf("%s\"wave%d\": [%llu, %llu, %llu, %llu, %llu, %llu]", w ? ", " : "", w,
               (unsigned long long)(t[w][1] - t[w][0]), (unsigned long long)(t[w][2] - t[w][0]),
               (unsigned long long)(t[w][3] - t[w][0]), (unsigned long long)(t[w][5] > t[w][0] ? t[w][5] - t[w][0] : 0),
               (unsigned long long)(t[w][6] > t[w][0] ? t[w][6] - t[w][0] : 0),
               (unsigned long long)(t[w][7] > t[w][0] ? t[w][7] - t[w][0] : 0));
    printf("}, \"wave0_end\": %llu, \"probes\": \"waves 0/1: table built, chain done, after the barrier; waves 2/3: "
           "hash/e/addr done, comb half done, after the barrier, all done, low-window chain start, its end; wave0_end: verdict written\"}\n",
           (unsigned long long)(t[0][4] - t[0][0]));
    return 0;
}
