// keccakcoop_check.hip -- the cooperative Keccak-f (hash_device.h KeccakCoop) against the one-lane
// keccak_f1600 on random states, plus probes of the cross-lane primitives it uses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../csrc/hash_device.h"
using namespace bcosgpu;

__global__ void probe(uint32_t* o) {
    const uint32_t l = threadIdx.x;
    o[l] = KeccakCoop::from_row1(l + 1000);
    o[64 + l] = KeccakCoop::from_row0(l + 1000);
    o[128 + l] = KeccakCoop::dpp<KeccakCoop::kR10>(l + 1000);
    o[192 + l] = KeccakCoop::dpp<KeccakCoop::kL10>(l + 1000);
}

// one state per 32-lane group: lane (x, y) loads word x + 5y of state g
__global__ void check(const uint64_t* st, uint64_t* out_coop, uint64_t* out_ref) {
    const KeccakCoop kc;
    const int lane = threadIdx.x & 63, grp = (blockIdx.x * (blockDim.x / 32)) + threadIdx.x / 32;
    const uint64_t* s = st + 25 * grp;
    uint32_t lo = 0, hi = 0;
    if (kc.gl < 25) {
        lo = static_cast<uint32_t>(s[kc.gl]);
        hi = static_cast<uint32_t>(s[kc.gl] >> 32);
    }
    kc.permute(lo, hi);
    if (kc.gl < 25) out_coop[25 * grp + kc.gl] = (static_cast<uint64_t>(hi) << 32) | lo;
    if ((lane & 31) == 0) {
        uint64_t a[25];
        for (int i = 0; i < 25; ++i) a[i] = s[i];
        keccak_f1600(a);
        for (int i = 0; i < 25; ++i) out_ref[25 * grp + i] = a[i];
    }
}

// s_memtime cycles of `reps` back-to-back permutations, cooperative vs one lane (a lone wave per SIMD)
__global__ void timing(uint64_t* cyc, int reps, uint64_t* sink) {
    const KeccakCoop kc;
    uint32_t lo = threadIdx.x, hi = threadIdx.x * 7u;
    uint64_t t0 = clock64();
    for (int r = 0; r < reps; ++r) kc.permute(lo, hi);
    uint64_t t1 = clock64();
    uint64_t a[25];
    for (int i = 0; i < 25; ++i) a[i] = lo + i;
    uint64_t t2 = clock64();
    for (int r = 0; r < reps; ++r) keccak_f1600(a);
    uint64_t t3 = clock64();
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / reps;
        cyc[1] = (t3 - t2) / reps;
    }
    sink[threadIdx.x] = lo ^ hi ^ a[0] ^ a[24];
}

int main() {
    uint32_t* dp;
    if (hipMalloc(&dp, 256 * 4) != hipSuccess) return 77;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dp);
    std::vector<uint32_t> p(256);
    (void)hipMemcpy(p.data(), dp, 1024, hipMemcpyDeviceToHost);
    const char* nm[4] = {"from_row1", "from_row0", "row_shl10", "row_shr10"};
    for (int k = 0; k < 4; ++k) {
        printf("%s:", nm[k]);
        for (int i = 0; i < 34; ++i) printf(" %d", (int)p[64 * k + i] - 1000);
        printf("\n");
    }
    const int G = 64;
    std::vector<uint64_t> st(25 * G), a(25 * G), b(25 * G);
    uint64_t x = 88172645463325252ull;
    for (auto& v : st) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    uint64_t *ds, *da, *db;
    (void)hipMalloc(&ds, st.size() * 8); (void)hipMalloc(&da, st.size() * 8); (void)hipMalloc(&db, st.size() * 8);
    (void)hipMemcpy(ds, st.data(), st.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check, dim3(G / 8), dim3(256), 0, 0, ds, da, db);
    (void)hipMemcpy(a.data(), da, a.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), db, b.size() * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 25 * G; ++i) bad += a[i] != b[i];
    uint64_t *dc, *dk;
    (void)hipMalloc(&dc, 16); (void)hipMalloc(&dk, 64 * 8);
    hipLaunchKernelGGL(timing, dim3(1), dim3(64), 0, 0, dc, 50, dk);
    uint64_t c[2];
    (void)hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
    printf("{\"states\": %d, \"mismatched_words\": %d, \"cycles_per_perm_coop\": %llu, \"cycles_per_perm_one_lane\": %llu}\n",
           G, bad, (unsigned long long)c[0], (unsigned long long)c[1]);
    return bad ? 1 : 0;
}
