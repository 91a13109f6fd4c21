// climbprobe.hip -- per-workgroup timelines (s_memrealtime, 10 ns ticks) of merkle_climb_kernel on a
// latency-sized narrow tree (default 100k leaves, width 2, Keccak: `climbprobe N WIDTH`): when each
// in-workgroup level ends (max / mean over workgroups), when the in-workgroup levels end, and for the
// workgroup that produced the root, when each climb step starts (after its arrival) and ends -- to see
// where the one-launch time goes.  Also the mean per-root time of 400 back-to-back launches.
#define BCOSGPU_MERKLE_PROBE 1
#include "../csrc/hash_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    using namespace bcosgpu;
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000;
    const int width = argc > 2 ? atoi(argv[2]) : 2;
    std::vector<uint8_t> leaves(n * 32);
    uint32_t x = 11;
    for (auto& b : leaves) b = (x = x * 1103515245u + 12345u) >> 24;
    uint64_t nodes = 0;
    for (uint64_t m = n; m > 1;) { m = (m + width - 1) / width; nodes += m + 1; }
    uint8_t *dl, *dt, *dr;
    if (hipMalloc(&dl, leaves.size()) != hipSuccess) return 77;
    (void)hipMalloc(&dt, 32 * (nodes + 2));
    (void)hipMalloc(&dr, 32);
    (void)hipMemcpy(dl, leaves.data(), leaves.size(), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 50; ++rep) launch_merkle(KECCAK256, width, dl, n, dt, dr, 0);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 400;
    (void)hipEventRecord(e0, 0);
    for (int rep = 0; rep < reps; ++rep) launch_merkle(KECCAK256, width, dl, n, dt, dr, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    static uint64_t mp[4096][40];
    std::memset(mp, 0, sizeof(mp));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_mp), mp, sizeof(mp));
    launch_merkle(KECCAK256, width, dl, n, dt, dr, 0);  // the stamps below are of this lone launch
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(mp, HIP_SYMBOL(g_mp), sizeof(mp));
    int wgs = 0;
    while (wgs < 4096 && mp[wgs][0]) ++wgs;
    uint64_t t0 = ~0ull;
    for (int b = 0; b < wgs; ++b) t0 = mp[b][0] < t0 ? mp[b][0] : t0;
    printf("{\"n\": %llu, \"width\": %d, \"ms_per_root\": %.4f, \"workgroups\": %d, ", (unsigned long long)n, width, ms / reps, wgs);
    auto stat = [&](int k, const char* name, bool comma) {
        uint64_t mx = 0, sum = 0;
        int cnt = 0;
        for (int b = 0; b < wgs; ++b)
            if (mp[b][k]) {
                const uint64_t v = mp[b][k] - t0;
                mx = v > mx ? v : mx;
                sum += v;
                ++cnt;
            }
        printf("\"%s\": [%.2f, %.2f]%s", name, cnt ? sum / 100.0 / cnt : 0.0, mx / 100.0, comma ? ", " : "");
    };
    stat(0, "start_mean_max_us", true);
    char nm[32];
    for (int l = 0; l < 19; ++l) {
        bool any = false;
        for (int b = 0; b < wgs; ++b) any = any || mp[b][20 + l];
        if (!any) break;
        snprintf(nm, sizeof(nm), "wg_level%d_end_us", l + 1);
        stat(20 + l, nm, true);
    }
    stat(1, "wg_levels_end_us", true);
    int root = -1, most = 0;
    for (int b = 0; b < wgs; ++b) {
        int c = 0;
        for (int k = 2; k < 20; ++k) c += mp[b][k] != 0;
        if (c > most) { most = c; root = b; }
    }
    printf("\"root_wg\": %d, \"root_wg_start_us\": %.2f, \"root_wg_levels_end_us\": %.2f, \"climb_us\": [", root,
           root >= 0 ? (mp[root][0] - t0) / 100.0 : 0.0, root >= 0 ? (mp[root][1] - t0) / 100.0 : 0.0);
    for (int k = 2; root >= 0 && k < 20 && mp[root][k]; ++k) printf("%s%.2f", k > 2 ? ", " : "", (mp[root][k] - t0) / 100.0);
    printf("]}\n");
    return 0;
}
