// keccakpair_check.hip -- the lane-pair Keccak (hash_device.h KeccakPair) against the one-lane
// keccak_f1600 / keccak256_msg on random states and messages, and the cycles of one permutation on a
// lone wave for the three variants (one lane, lane pair, 25-lane cooperative) and of one SM3
// compression (one lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../csrc/hash_device.h"
using namespace bcosgpu;

// one state per lane pair: the even lane loads the low halves, the odd lane the high halves
__global__ void check_perm(const uint64_t* st, uint64_t* out_pair, uint64_t* out_ref) {
    const KeccakPair kp;
    const int t = blockIdx.x * blockDim.x + threadIdx.x, s = t >> 1, half = t & 1;
    uint32_t a[25];
    for (int i = 0; i < 25; ++i) a[i] = static_cast<uint32_t>(st[25 * s + i] >> (32 * half));
    kp.permute(a);
    uint32_t* o = reinterpret_cast<uint32_t*>(out_pair + 25 * s);
    for (int i = 0; i < 25; ++i) o[2 * i + half] = a[i];
    if (!half) {
        uint64_t r[25];
        for (int i = 0; i < 25; ++i) r[i] = st[25 * s + i];
        keccak_f1600(r);
        for (int i = 0; i < 25; ++i) out_ref[25 * s + i] = r[i];
    }
}

// message m of length 4 m bytes (m = 0 .. NMSG - 1) from buf + 64 m
__global__ void check_msg(const uint8_t* buf, int nmsg, uint32_t* out_pair, uint32_t* out_ref) {
    const KeccakPair kp;
    const int t = blockIdx.x * blockDim.x + threadIdx.x, m = t >> 1, half = t & 1;
    if (m >= nmsg) return;  // whole pairs leave together
    const uint8_t* msg = buf + 64 * m;
    const uint32_t len = 4u * m;
    uint32_t d[4];
    kp.hash(msg, len, d);
    for (int j = 0; j < 4; ++j) out_pair[8 * m + 2 * j + half] = d[j];
    if (!half) {
        uint32_t r[8];
        keccak256_msg(AlignedReader(msg, len), len, r);
        for (int j = 0; j < 8; ++j) out_ref[8 * m + j] = r[j];
    }
}

__global__ void timing(uint64_t* cyc, int reps, uint64_t* sink) {
    const KeccakPair kp;
    const KeccakCoop kc;
    uint32_t a[25];
    for (int i = 0; i < 25; ++i) a[i] = threadIdx.x * 31u + i;
    uint64_t t0 = clock64();
    for (int r = 0; r < reps; ++r) kp.permute(a);
    uint64_t t1 = clock64();
    uint64_t s[25];
    for (int i = 0; i < 25; ++i) s[i] = a[i] + i;
    uint64_t t2 = clock64();
    for (int r = 0; r < reps; ++r) keccak_f1600(s);
    uint64_t t3 = clock64();
    uint32_t lo = static_cast<uint32_t>(s[0]), hi = static_cast<uint32_t>(s[1]);
    uint64_t t4 = clock64();
    for (int r = 0; r < reps; ++r) kc.permute(lo, hi);
    uint64_t t5 = clock64();
    uint32_t V[8], W[16];
    for (int i = 0; i < 8; ++i) V[i] = lo + i;
    for (int i = 0; i < 16; ++i) W[i] = hi * 3u + i;
    uint64_t t6 = clock64();
    for (int r = 0; r < reps; ++r) sm3_compress(V, W);
    uint64_t t7 = clock64();
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / reps;
        cyc[1] = (t3 - t2) / reps;
        cyc[2] = (t5 - t4) / reps;
        cyc[3] = (t7 - t6) / reps;
    }
    uint32_t x = lo ^ hi ^ V[0] ^ V[7];
    for (int i = 0; i < 25; ++i) x ^= a[i] ^ static_cast<uint32_t>(s[i]);
    sink[threadIdx.x] = x;
}

int main() {
    const int S = 256;  // states
    std::vector<uint64_t> st(25 * S), a(25 * S), b(25 * S);
    uint64_t x = 88172645463325252ull;
    for (auto& v : st) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    uint64_t *ds, *da, *db;
    if (hipMalloc(&ds, st.size() * 8) != hipSuccess) return 77;
    (void)hipMalloc(&da, st.size() * 8); (void)hipMalloc(&db, st.size() * 8);
    (void)hipMemcpy(ds, st.data(), st.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check_perm, dim3(2 * S / 256), dim3(256), 0, 0, ds, da, db);
    (void)hipMemcpy(a.data(), da, a.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), db, b.size() * 8, hipMemcpyDeviceToHost);
    int bad_perm = 0;
    for (int i = 0; i < 25 * S; ++i) bad_perm += a[i] != b[i];

    const int NM = 160;  // lengths 0 .. 636 bytes (5 blocks), every multiple of 4
    std::vector<uint8_t> buf(64 * NM + 1024);
    for (auto& v : buf) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = static_cast<uint8_t>(x); }
    // messages overlap in buf (message m starts at 64 m, runs 4 m bytes): fine, reads only
    uint8_t* dbuf;
    uint32_t *dp, *dr;
    (void)hipMalloc(&dbuf, buf.size());
    (void)hipMalloc(&dp, NM * 32); (void)hipMalloc(&dr, NM * 32);
    (void)hipMemcpy(dbuf, buf.data(), buf.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check_msg, dim3((2 * NM + 255) / 256), dim3(256), 0, 0, dbuf, NM, dp, dr);
    std::vector<uint32_t> p(8 * NM), r(8 * NM);
    (void)hipMemcpy(p.data(), dp, NM * 32, hipMemcpyDeviceToHost);
    (void)hipMemcpy(r.data(), dr, NM * 32, hipMemcpyDeviceToHost);
    int bad_msg = 0;
    for (int i = 0; i < 8 * NM; ++i) bad_msg += p[i] != r[i];

    uint64_t *dc, *dk;
    (void)hipMalloc(&dc, 32); (void)hipMalloc(&dk, 64 * 8);
    hipLaunchKernelGGL(timing, dim3(1), dim3(64), 0, 0, dc, 40, dk);
    uint64_t c[4];
    (void)hipMemcpy(c, dc, 32, hipMemcpyDeviceToHost);
    printf("{\"states\": %d, \"perm_mismatched_words\": %d, \"messages\": %d, \"msg_mismatched_words\": %d, "
           "\"cycles_per_perm_pair\": %llu, \"cycles_per_perm_one_lane\": %llu, \"cycles_per_perm_coop25\": %llu, "
           "\"cycles_per_sm3_compression\": %llu}\n",
           S, bad_perm, NM, bad_msg, (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
           (unsigned long long)c[3]);
    return bad_perm || bad_msg ? 1 : 0;
}
