// fusedprobe.hip -- per-wave timelines (s_memrealtime, 10 ns ticks) of merkle_fused_kernel at merkleBench
// size (100k leaves, width 16; or `fusedprobe N WIDTH`) for Keccak and SM3: when level 0, the in-wave
// levels and each climbed level end (the start and end of each climbed level's hash), relative to the
// earliest wave start; to see where the one-launch time goes.  Also the mean per-root time of 400
// back-to-back launches.
#define BCOSGPU_MERKLE_PROBE 1
#include "../csrc/hash_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    using namespace bcosgpu;
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000;
    const int width = argc > 2 ? atoi(argv[2]) : 16;
    std::vector<uint8_t> leaves(n * 32);
    uint32_t x = 7;
    for (auto& b : leaves) b = (x = x * 1103515245u + 12345u) >> 24;
    uint64_t nodes = 0;
    for (uint64_t m = n; m > 1;) { m = (m + width - 1) / width; nodes += m + 1; }
    uint8_t *dl, *dt, *dr;
    if (hipMalloc(&dl, leaves.size()) != hipSuccess) return 77;
    (void)hipMalloc(&dt, 32 * (nodes + 2));
    (void)hipMalloc(&dr, 32);
    (void)hipMemcpy(dl, leaves.data(), leaves.size(), hipMemcpyHostToDevice);
    setenv("BCOSGPU_MERKLE_FUSED", "1", 1);
    for (int h : {KECCAK256, SM3}) {
        for (int rep = 0; rep < 50; ++rep) launch_merkle(h, width, dl, n, dt, dr, 0);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;  // back-to-back launches: the per-root time the bench's Merkle legs report
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const int reps = 400;
        (void)hipEventRecord(e0, 0);
        for (int rep = 0; rep < reps; ++rep) launch_merkle(h, width, dl, n, dt, dr, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        launch_merkle(h, width, dl, n, dt, dr, 0);  // the stamps below are of this lone launch
        (void)hipDeviceSynchronize();
        static uint64_t mp[4096][40];
        (void)hipMemcpyFromSymbol(mp, HIP_SYMBOL(g_mp), sizeof(mp));
        uint64_t S = 1;  // level-1 nodes per wave (launch_merkle_fused: width^a <= 32 for Keccak, <= 64 for SM3)
        while (S * width <= (h == KECCAK256 ? 32u : 64u)) S *= width;
        const uint64_t waves = ((n + width - 1) / width + S - 1) / S;
        uint64_t t0 = ~0ull, l0max = 0, innermax = 0, l0sum = 0;
        for (uint64_t b = 0; b < waves && b < 4096; ++b) t0 = mp[b][0] < t0 ? mp[b][0] : t0;
        uint64_t smax = 0;
        for (uint64_t b = 0; b < waves && b < 4096; ++b) {
            smax = mp[b][0] - t0 > smax ? mp[b][0] - t0 : smax;
            l0max = mp[b][1] - t0 > l0max ? mp[b][1] - t0 : l0max;
            innermax = mp[b][2] - t0 > innermax ? mp[b][2] - t0 : innermax;
            l0sum += mp[b][1] - mp[b][0];
        }
        printf("{\"hasher\": %d, \"n\": %llu, \"width\": %d, \"ms_per_root\": %.4f, \"waves\": %llu, \"last_start_us\": %.2f, \"level0_mean_us\": %.2f, \"level0_end_max_us\": %.2f, "
               "\"inner_end_max_us\": %.2f, \"climb\": [", h, (unsigned long long)n, width, ms / reps, (unsigned long long)waves, smax / 100.0,
               l0sum / 100.0 / waves, l0max / 100.0, innermax / 100.0);
        // the wave that wrote the root: the one with the most climb stamps of this launch
        for (int k = 3; k < 40; ++k) {
            uint64_t best = 0;
            for (uint64_t b = 0; b < waves && b < 4096; ++b)
                if (mp[b][k] > mp[b][0] && mp[b][k] >= t0 && mp[b][k] - t0 < 100000 && mp[b][k] - t0 > best) best = mp[b][k] - t0;
            printf("%s%.2f", k > 3 ? ", " : "", best / 100.0);
        }
        printf("]}\n");
    }
    return 0;
}
