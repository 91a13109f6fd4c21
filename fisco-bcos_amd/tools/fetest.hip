// fetest.hip -- field-arithmetic vectors for tests/test_gpu_field.py: reads lines "op a b" (hex,
// 256-bit, op in add/sub/mul/sqr/norm/shl1/shl2/shl3/mul3) from stdin, evaluates them with FieldK1 on the GPU (one
// vector per lane), prints the canonical result per line.  Covers the rare carry/borrow tails of
// the k1_add/k1_sub asm that random inputs almost never reach.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include "../csrc/fe.h"

using namespace bcosgpu;

__global__ void k(const uint32_t* in, const int* op, int n, uint32_t* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe a, b, r;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        a.v[w] = in[16 * i + w];
        b.v[w] = in[16 * i + 8 + w];
    }
    switch (op[i]) {
        case 0: FieldK1::add(r, a, b); break;
        case 1: FieldK1::sub(r, a, b); break;
        case 2: FieldK1::mul(r, a, b); break;
        case 3: FieldK1::sqr(r, a); break;
        case 5: FieldK1::shl<1>(r, a); break;
        case 6: FieldK1::shl<2>(r, a); break;
        case 7: FieldK1::shl<3>(r, a); break;
        case 8: FieldK1::mul3(r, a); break;
        default: fe_copy(r, a); break;
    }
    FieldK1::normalize(r);
#pragma unroll
    for (int w = 0; w < 8; ++w) out[8 * i + w] = r.v[w];
}

static void parse(const char* h, uint32_t* w) {
    char buf[65];
    const size_t len = strlen(h) < 64 ? strlen(h) : 64;
    memset(buf, '0', 64);
    memcpy(buf + 64 - len, h + strlen(h) - len, len);
    buf[64] = 0;
    for (int q = 0; q < 8; ++q) {
        char part[9];
        memcpy(part, buf + 8 * (7 - q), 8);
        part[8] = 0;
        w[q] = static_cast<uint32_t>(strtoul(part, nullptr, 16));
    }
}

int main() {
    std::vector<uint32_t> in;
    std::vector<int> ops;
    char op[8], a[80], b[80];
    while (scanf("%7s %79s %79s", op, a, b) == 3) {
        uint32_t w[16];
        parse(a, w);
        parse(b, w + 8);
        in.insert(in.end(), w, w + 16);
        const std::string o(op);
        ops.push_back(o == "add" ? 0 : o == "sub" ? 1 : o == "mul" ? 2 : o == "sqr" ? 3 : o == "shl1" ? 5
                      : o == "shl2" ? 6 : o == "shl3" ? 7 : o == "mul3" ? 8 : 4);
    }
    const int n = static_cast<int>(ops.size());
    if (!n) return 0;
    uint32_t *din, *dout;
    int* dop;
    if (hipMalloc(&din, in.size() * 4) != hipSuccess || hipMalloc(&dout, n * 32) != hipSuccess ||
        hipMalloc(&dop, n * 4) != hipSuccess ||
        hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dop, ops.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, din, dop, n, dout);
    std::vector<uint32_t> out(8 * n);
    if (hipMemcpy(out.data(), dout, n * 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int i = 0; i < n; ++i) {
        for (int q = 7; q >= 0; --q) printf("%08x", out[8 * i + q]);
        printf("\n");
    }
    return 0;
}
