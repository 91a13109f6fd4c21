// fe26test.hip -- GPU check of the fe26 device arithmetic (the inline-asm mul / sqr of fe_asm.h and the
// C++ linear ops) on deterministic operands; prints one line per case for tests/test_fe26.py-style
// checking with Python integers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../csrc/ec26.h"
using namespace bcosgpu;

__device__ uint32_t xs(uint64_t& s) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return static_cast<uint32_t>(s >> 11);
}
__global__ void k(uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s = 0x9e3779b97f4a7c15ull + i * 7919ull;
    fe26 a, b, r, q;
    const uint32_t m = (i % 4 == 0) ? 16u : (i % 4 == 1) ? 1u : (i % 4 == 2) ? 4u : 2u;
    for (int j = 0; j < 10; ++j) {
        const uint64_t bound = static_cast<uint64_t>(m) << (j == 9 ? 22 : 26);
        a.v[j] = static_cast<uint32_t>(((static_cast<uint64_t>(xs(s)) << 20) ^ xs(s)) % (bound + 1));
        b.v[j] = static_cast<uint32_t>(((static_cast<uint64_t>(xs(s)) << 20) ^ xs(s)) % (bound + 1));
    }
    fe26_mul(r, a, b);
    fe26_sqr(q, a);
    uint32_t* o = out + i * 40;
    for (int j = 0; j < 10; ++j) { o[j] = a.v[j]; o[10 + j] = b.v[j]; o[20 + j] = r.v[j]; o[30 + j] = q.v[j]; }
}
int main() {
    const int n = 4096;
    uint32_t* d;
    hipMalloc(&d, n * 40 * 4);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, n);
    uint32_t* h = new uint32_t[n * 40];
    hipMemcpy(h, d, n * 40 * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < 40; ++j) printf("%x%c", h[i * 40 + j], j == 39 ? '\n' : ' ');
    }
    return 0;
}
