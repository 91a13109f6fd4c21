// ecc_tables.hip -- comb tables of G (8-bit and 16-bit, both curves; the SM2 ones also in fp26's R' domain), their
// per-device registry and the tx-kernel selection policy.
#include "ecc_device.h"

namespace bcosgpu {

static std::mutex g_tab_mu;
static uint32_t* g_tab_k1[64];
static uint32_t* g_tab_sm2[64];
static uint32_t* g_wtab_k1[64];
static uint32_t* g_wtab_sm2[64];
static uint32_t* g_tab_sm2_26[64];   // the SM2 tables re-expressed in fp26's Montgomery domain (R = 2^286)
static uint32_t* g_wtab_sm2_26[64];

// ------------------------------------------------------------------ table construction
template <class C, class F>
__global__ __launch_bounds__(256) void comb_table_kernel(uint32_t* tab, int sm2) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= kCombWindows * kCombEntries) return;
    const int i = idx / kCombEntries;
    uint32_t b = static_cast<uint32_t>(idx % kCombEntries);
    if (b == 0) b = 1;  // unused slot: a valid point, never selected
    fe k;
#pragma unroll
    for (int q = 0; q < 8; ++q) k.v[q] = (q == (i >> 2)) ? (b << ((i & 3) * 8)) : 0u;
    Aff G;
    fe gx, gy;
    fe_set(gx, sm2 ? kSM2Gx : kK1Gx);
    fe_set(gy, sm2 ? kSM2Gy : kK1Gy);
    fe_copy(G.x, gx);
    fe_copy(G.y, gy);
    Jac acc, S;
    C::set_inf(acc);
#pragma unroll 1
    for (int bit = 255; bit >= 0; --bit) {
        C::dbl(acc, acc);
        const bool set = (k.v[7] >> 31) != 0u;
        shl1(k);
        C::madd(S, acc, G);
        C::cmov(acc, S, set);
    }
    Aff A;
    C::to_aff(A, acc);
    F::normalize(A.x);
    F::normalize(A.y);
    uint32_t* o = tab + static_cast<size_t>(idx) * 16;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        o[w] = A.x.v[w];
        o[8 + w] = A.y.v[w];
    }
}

// 16-bit comb entry (i, b) = lo * 2^(16 i) G + hi * 2^(16 i + 8) G (b = lo + 256 hi): one addition of
// two 8-bit-table entries and one inversion.  The two addends never coincide or cancel
// (lo - 256 hi != 0 mod n), and the madd is complete anyway.
template <class C, class F>
__global__ __launch_bounds__(256) void comb_wide_kernel(uint32_t* __restrict__ wide, const uint32_t* __restrict__ tab8) {
    const uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= static_cast<uint64_t>(kWideWindows) * kWideEntries) return;
    const int i = static_cast<int>(idx / kWideEntries);
    uint32_t b = static_cast<uint32_t>(idx % kWideEntries);
    if (b == 0) b = 1;  // unused slot: a valid point, never selected
    const uint32_t lo = b & 255u, hi = b >> 8;
    Aff A, B;
    load_aff16(A, tab8 + (static_cast<size_t>(2 * i) * kCombEntries + (lo ? lo : 1u)) * 16);
    load_aff16(B, tab8 + (static_cast<size_t>(2 * i + 1) * kCombEntries + (hi ? hi : 1u)) * 16);
    Aff R;
    if (lo && hi) {
        Jac P, S;
        C::from_aff(P, A);
        C::madd(S, P, B);
        C::to_aff(R, S);
        F::normalize(R.x);
        F::normalize(R.y);
    } else {
        R = lo ? A : B;
    }
    uint32_t* o = wide + idx * 16;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        o[w] = R.x.v[w];
        o[8 + w] = R.y.v[w];
    }
}

static TxKernelPolicy g_policy;
static bool g_policy_read = false;

static void read_policy_env() {
    if (g_policy_read) return;
    g_policy_read = true;
    if (const char* e = getenv("BCOSGPU_TXV_SPLIT")) g_policy.split = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : -1;
    if (const char* e = getenv("BCOSGPU_TXV_OCC")) g_policy.occ = (atoi(e) == 1 || atoi(e) == 2) ? atoi(e) : 0;
    if (const char* e = getenv("BCOSGPU_TXV_COOP")) g_policy.coop = atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : atoi(e) == 3 ? 3 : 2;
    if (const char* e = getenv("BCOSGPU_K1_F26")) g_policy.f26 = atoi(e) != 0;
}

void set_tx_kernel_policy(int split, int occ, int coop, int f26) {
    std::lock_guard<std::mutex> g(g_tab_mu);
    read_policy_env();
    g_policy.split = (split == 0 || split == 1) ? split : -1;
    g_policy.occ = (occ == 1 || occ == 2) ? occ : 0;
    g_policy.coop = coop == 0 ? 0 : coop == 1 ? 1 : coop == 3 ? 3 : 2;
    if (f26 == 0 || f26 == 1) g_policy.f26 = f26;
}

static void free_tables(uint32_t*& a, uint32_t*& b, uint32_t*& c, uint32_t*& d) {
    for (uint32_t** p : {&a, &b, &c, &d}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
}

// init: SM2 comb table entries (x || y, R = 2^256 Montgomery domain, canonical) -> fp26's R' = 2^286
// domain: the Montgomery product (R domain) with 2^286 mod p
__device__ __constant__ static const uint32_t kSm2RtoR26[8] = {0x40000000u, 0x0u, 0xc0000000u, 0x3fffffffu,
                                                               0x0u,        0x0u, 0x0u,        0x40000000u};
__global__ __launch_bounds__(256) void sm2_table_to_r26_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                               uint64_t entries) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= entries) return;
    fe c, x, y;
    fe_set(c, kSm2RtoR26);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        x.v[w] = src[i * 16 + w];
        y.v[w] = src[i * 16 + 8 + w];
    }
    FieldP2::mul(x, x, c);
    FieldP2::mul(y, y, c);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        dst[i * 16 + w] = x.v[w];
        dst[i * 16 + 8 + w] = y.v[w];
    }
}

// Builds the device's comb tables: the 8-bit ones (512 KiB per curve) always; the 16-bit ones (64 MiB
// per curve) unless `small` or their allocation fails -- the kernels then run the 8-bit comb.
int ecc_init_tables(int device, int small) {
    std::lock_guard<std::mutex> g(g_tab_mu);
    read_policy_env();
    if (device < 0 || device >= 64) return BCOSGPU_E_ARG;
    if (g_tab_k1[device] && g_tab_sm2[device]) return 0;
    if (const char* e = getenv("BCOSGPU_TABLES")) small = small || std::strcmp(e, "small") == 0;
    uint32_t *k1 = nullptr, *sm2 = nullptr, *wk1 = nullptr, *wsm2 = nullptr;
    if (hipMalloc(&k1, kTabWords * 4) != hipSuccess || hipMalloc(&sm2, kTabWords * 4) != hipSuccess) {
        (void)hipGetLastError();
        free_tables(k1, sm2, wk1, wsm2);
        return BCOSGPU_E_HIP;
    }
    const int n = kCombWindows * kCombEntries;
    hipLaunchKernelGGL((comb_table_kernel<CurveK1, FieldK1>), dim3((n + 255) / 256), dim3(256), 0, 0, k1, 0);
    hipLaunchKernelGGL((comb_table_kernel<CurveSM2, FieldP2>), dim3((n + 255) / 256), dim3(256), 0, 0, sm2, 1);
    if (!small && (hipMalloc(&wk1, kWideTabWords * 4) != hipSuccess ||
                   hipMalloc(&wsm2, kWideTabWords * 4) != hipSuccess)) {
        (void)hipGetLastError();  // not enough memory for the wide tables: run on the 8-bit ones
        if (wk1) (void)hipFree(wk1);
        if (wsm2) (void)hipFree(wsm2);
        wk1 = wsm2 = nullptr;
    }
    if (wk1) {
        const unsigned gw = static_cast<unsigned>((static_cast<uint64_t>(kWideWindows) * kWideEntries + 255) / 256);
        hipLaunchKernelGGL((comb_wide_kernel<CurveK1, FieldK1>), dim3(gw), dim3(256), 0, 0, wk1, k1);
        hipLaunchKernelGGL((comb_wide_kernel<CurveSM2, FieldP2>), dim3(gw), dim3(256), 0, 0, wsm2, sm2);
    }
    uint32_t *sm2r = nullptr, *wsm2r = nullptr;
    if (hipMalloc(&sm2r, kTabWords * 4) != hipSuccess) {
        (void)hipGetLastError();
        free_tables(k1, sm2, wk1, wsm2);
        return BCOSGPU_E_HIP;
    }
    {
        const uint64_t ent = kTabWords / 16;
        hipLaunchKernelGGL(sm2_table_to_r26_kernel, dim3(static_cast<unsigned>((ent + 255) / 256)), dim3(256), 0, 0,
                           sm2r, sm2, ent);
    }
    if (wsm2) {
        if (hipMalloc(&wsm2r, kWideTabWords * 4) == hipSuccess) {
            const uint64_t ent = kWideTabWords / 16;
            hipLaunchKernelGGL(sm2_table_to_r26_kernel, dim3(static_cast<unsigned>((ent + 255) / 256)), dim3(256), 0,
                               0, wsm2r, wsm2, ent);
        } else {  // no room for the R'-domain copy of the wide SM2 table: every SM2 kernel on the 8-bit ones
            (void)hipGetLastError();
            wsm2r = nullptr;
        }
    }
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        free_tables(k1, sm2, wk1, wsm2);
        if (sm2r) (void)hipFree(sm2r);
        if (wsm2r) (void)hipFree(wsm2r);
        return BCOSGPU_E_HIP;
    }
    g_tab_sm2_26[device] = sm2r;
    g_wtab_sm2_26[device] = wsm2r;
    g_tab_k1[device] = k1;
    g_tab_sm2[device] = sm2;
    g_wtab_k1[device] = wk1;
    g_wtab_sm2[device] = wsm2;
    return 0;
}

TxKernelPolicy tx_policy() {
    std::lock_guard<std::mutex> g(g_tab_mu);
    return g_policy;
}

static int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    return dev;
}

// The comb tables of the current device: the 16-bit ones when present (*bits = 16), else the 8-bit
// ones (*bits = 8).
int tables(const uint32_t** k1, const uint32_t** sm2, int* bits) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_k1[dev]) return BCOSGPU_E_NODEV;  // bcosgpu_init(dev) not called
    const bool wide = g_wtab_k1[dev] != nullptr;
    *k1 = wide ? g_wtab_k1[dev] : g_tab_k1[dev];
    *sm2 = wide ? g_wtab_sm2[dev] : g_tab_sm2[dev];
    *bits = wide ? kWideBits : 8;
    return 0;
}
// the SM2 comb table in fp26's R' domain: the 16-bit one when present, else the 8-bit one
int tables_sm2_26(const uint32_t** tab, int* bits) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_sm2_26[dev]) return BCOSGPU_E_NODEV;
    const bool wide = g_wtab_sm2_26[dev] != nullptr;
    *tab = wide ? g_wtab_sm2_26[dev] : g_tab_sm2_26[dev];
    *bits = wide ? kWideBits : 8;
    return 0;
}
// 8-bit comb tables
int tables8(const uint32_t** k1, const uint32_t** sm2) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return BCOSGPU_E_NODEV;
    if (!g_tab_k1[dev]) return BCOSGPU_E_NODEV;
    *k1 = g_tab_k1[dev];
    *sm2 = g_tab_sm2[dev];
    return 0;
}
int tables8_sm2_26(const uint32_t** tab) {
    const int dev = current_device();
    if (dev < 0 || !g_tab_sm2_26[dev]) return BCOSGPU_E_NODEV;
    *tab = g_tab_sm2_26[dev];
    return 0;
}
}  // namespace bcosgpu
