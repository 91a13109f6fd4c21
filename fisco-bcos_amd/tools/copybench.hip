// copybench.hip -- host<->device copy costs that shape the host-pointer batch paths (api.hip, multi.hip):
// pageable vs pinned hipMemcpyAsync bandwidth and per-call latency, host memcpy into pinned memory at
// 1..8 threads, hipHostRegister cost, and whether a pageable copy on one stream overlaps a kernel on
// another.  Prints one JSON object.  GPU tool, not part of the product.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ~`iters` dependent integer ops per lane: a kernel of known length on a few CUs
__global__ void spin_kernel(uint32_t* out, uint32_t iters) {
    uint32_t x = threadIdx.x + 1;
    for (uint32_t i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

static double time_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind k, hipStream_t s, int reps) {
    CK(hipMemcpyAsync(dst, src, bytes, k, s));
    CK(hipStreamSynchronize(s));
    const double t0 = now();
    for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dst, src, bytes, k, s));
    CK(hipStreamSynchronize(s));
    return (now() - t0) / reps;
}

static void par_memcpy(uint8_t* dst, const uint8_t* src, size_t bytes, int threads) {
    if (threads <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (bytes + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const size_t lo = std::min(bytes, per * t), hi = std::min(bytes, per * (t + 1));
        th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
    }
    for (auto& x : th) x.join();
}

int main() {
    CK(hipSetDevice(0));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    const size_t big = 256ull << 20;
    std::vector<uint8_t> pageable(big, 1), pageable_out(big, 0);
    uint8_t *pinned = nullptr, *dev = nullptr;
    CK(hipHostMalloc(&pinned, big, hipHostMallocDefault));
    std::memset(pinned, 2, big);
    CK(hipMalloc(&dev, big));
    uint32_t* spin_out;
    CK(hipMalloc(&spin_out, 4096));
    const size_t sizes[] = {4096, 65536, 530000, 2300000, 27000000, 216000000};
    std::printf("{\"copies\":[");
    bool first = true;
    for (size_t sz : sizes) {
        const int reps = sz < 1000000 ? 200 : sz < 50000000 ? 20 : 4;
        const double h2d_pg = time_copy(dev, pageable.data(), sz, hipMemcpyHostToDevice, s0, reps);
        const double d2h_pg = time_copy(pageable_out.data(), dev, sz, hipMemcpyDeviceToHost, s0, reps);
        const double h2d_pin = time_copy(dev, pinned, sz, hipMemcpyHostToDevice, s0, reps);
        const double d2h_pin = time_copy(pinned, dev, sz, hipMemcpyDeviceToHost, s0, reps);
        std::printf("%s{\"bytes\":%zu,\"h2d_pageable_us\":%.2f,\"d2h_pageable_us\":%.2f,\"h2d_pinned_us\":%.2f,"
                    "\"d2h_pinned_us\":%.2f,\"h2d_pageable_GBs\":%.2f,\"h2d_pinned_GBs\":%.2f,\"d2h_pageable_GBs\":%.2f,"
                    "\"d2h_pinned_GBs\":%.2f}",
                    first ? "" : ",", sz, h2d_pg * 1e6, d2h_pg * 1e6, h2d_pin * 1e6, d2h_pin * 1e6, sz / h2d_pg / 1e9,
                    sz / h2d_pin / 1e9, sz / d2h_pg / 1e9, sz / d2h_pin / 1e9);
        first = false;
    }
    std::printf("],\"host_memcpy\":[");
    first = true;
    for (size_t sz : {(size_t)2300000, (size_t)27000000, (size_t)216000000}) {
        for (int t : {1, 2, 4, 8}) {
            par_memcpy(pinned, pageable.data(), sz, t);
            const int reps = sz < 50000000 ? 20 : 3;
            const double t0 = now();
            for (int r = 0; r < reps; ++r) par_memcpy(pinned, pageable.data(), sz, t);
            const double dt = (now() - t0) / reps;
            std::printf("%s{\"bytes\":%zu,\"threads\":%d,\"us\":%.2f,\"GBs\":%.2f}", first ? "" : ",", sz, t, dt * 1e6,
                        sz / dt / 1e9);
            first = false;
        }
    }
    std::printf("],\"register\":[");
    first = true;
    for (size_t sz : {(size_t)2300000, (size_t)27000000, (size_t)216000000}) {
        std::vector<uint8_t> buf(sz + 4096, 3);
        const double t0 = now();
        CK(hipHostRegister(buf.data(), sz, hipHostRegisterDefault));
        const double t1 = now();
        void* dp = nullptr;
        CK(hipHostGetDevicePointer(&dp, buf.data(), 0));
        const double h2d = time_copy(dev, buf.data(), sz, hipMemcpyHostToDevice, s0, 3);
        const double t2 = now();
        CK(hipHostUnregister(buf.data()));
        const double t3 = now();
        std::printf("%s{\"bytes\":%zu,\"register_us\":%.1f,\"unregister_us\":%.1f,\"h2d_registered_GBs\":%.2f}",
                    first ? "" : ",", sz, (t1 - t0) * 1e6, (t3 - t2) * 1e6, sz / h2d / 1e9);
        first = false;
    }
    // overlap: a ~20 ms kernel on s0, a 27 MB pageable (then pinned) H2D on s1 issued right after
    std::printf("],\"overlap\":{");
    const uint32_t iters = 4000000;
    hipLaunchKernelGGL(spin_kernel, dim3(4), dim3(64), 0, s0, spin_out, iters);
    CK(hipStreamSynchronize(s0));
    double t0 = now();
    hipLaunchKernelGGL(spin_kernel, dim3(4), dim3(64), 0, s0, spin_out, iters);
    CK(hipStreamSynchronize(s0));
    const double kt = now() - t0;
    const size_t osz = 27000000;
    const double c_pg = time_copy(dev, pageable.data(), osz, hipMemcpyHostToDevice, s1, 1);
    t0 = now();
    hipLaunchKernelGGL(spin_kernel, dim3(4), dim3(64), 0, s0, spin_out, iters);
    const double t_issue0 = now();
    CK(hipMemcpyAsync(dev, pageable.data(), osz, hipMemcpyHostToDevice, s1));
    const double t_ret_pg = now();
    CK(hipStreamSynchronize(s1));
    const double t_copy_pg = now();
    CK(hipStreamSynchronize(s0));
    const double t_all_pg = now();
    hipLaunchKernelGGL(spin_kernel, dim3(4), dim3(64), 0, s0, spin_out, iters);
    const double u0 = now();
    CK(hipMemcpyAsync(dev, pinned, osz, hipMemcpyHostToDevice, s1));
    const double u_ret = now();
    CK(hipStreamSynchronize(s1));
    const double u_copy = now();
    CK(hipStreamSynchronize(s0));
    const double u_all = now();
    std::printf("\"kernel_ms\":%.3f,\"copy_alone_ms\":%.3f,\"pageable\":{\"issue_return_ms\":%.3f,\"copy_done_ms\":%.3f,"
                "\"all_done_ms\":%.3f},\"pinned\":{\"issue_return_ms\":%.3f,\"copy_done_ms\":%.3f,\"all_done_ms\":%.3f}}",
                kt * 1e3, c_pg * 1e3, (t_ret_pg - t_issue0) * 1e3, (t_copy_pg - t0) * 1e3, (t_all_pg - t0) * 1e3,
                (u_ret - u0) * 1e3, (u_copy - u0) * 1e3, (u_all - u0) * 1e3);
    std::printf("}\n");
    return 0;
}
