// api.hip -- the C ABI (include/bcos_gpu.h): argument checks, per-device workspaces for the
// host-pointer entry points, and the wedpr-shaped single-call shims.  No exceptions cross the ABI.
#include <atomic>
#include <mutex>
#include <string>
#include <vector>
#include <cstring>
#include "engine.h"

using namespace bcosgpu;

namespace {

thread_local std::string g_err;
int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_err(hipError_t e, const char* what) {
    return set_err(BCOSGPU_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_OK(call)                                   \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) return hip_err(e_, #call); \
    } while (0)

// Grow-only device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Grow-only pinned host buffer (staging for packers that write straight into DMA-able memory).
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// One workspace per device for the synchronous host-pointer API; the mutex makes those entry
// points safe to call from the reference's concurrent verifier pools (TxPool.h:48-49).
struct Workspace {
    std::mutex mu;
    bool ready = false;
    hipStream_t stream = nullptr;
    DevBuf b[8];
    HostBuf h[2];
};
std::mutex g_mu;
std::vector<Workspace*> g_ws;
std::atomic<bool> g_ready[64];  // device initialised (tables built): the single-call fast path

int current_device(int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return set_err(BCOSGPU_E_NODEV, "no HIP device visible");
    }
    HIP_OK(hipGetDevice(dev));
    return 0;
}

int get_ws(Workspace** out) {
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    rc = bcosgpu_init(dev);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(g_mu);
    *out = g_ws[dev];
    return 0;
}

inline hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

int init_device(int device, int flags);

// The explicit-device entry points: initialise `device` once, without changing the calling thread's
// current device.
int ready_device(int device) {
    if (device >= 0 && device < 64 && g_ready[device].load(std::memory_order_acquire)) return 0;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) {
        (void)hipGetLastError();
        prev = -1;
    }
    const int rc = init_device(device, 0);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return rc;
}

// A host-pointer signature call as a coalesced job (coalesce.hip) on `device`.
int run_job(int device, SigJob& job) {
    int rc = ready_device(device);
    if (rc) return rc;
    rc = coalesced_run(device, job);
    return rc ? set_err(rc, job.err) : 0;
}

int calling_device(int* dev) {
    int rc = current_device(dev);
    return rc ? rc : ready_device(*dev);
}

}  // namespace

// for the device-set entry points (multi.hip)
namespace bcosgpu {
int api_set_err(int code, const std::string& msg) { return set_err(code, msg); }
int api_ready_device(int device) { return ready_device(device); }
int api_run_job(int device, SigJob& job) { return run_job(device, job); }
}  // namespace bcosgpu

extern "C" {

int bcosgpu_version(void) { return BCOSGPU_VERSION; }

int bcosgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

const char* bcosgpu_last_error(void) { return g_err.c_str(); }

uint64_t bcosgpu_merkle_size(uint64_t n, int width) {
    if (width < 2) return 0;
    return n == 1 ? 1 : merkle_size(n, width);
}

int bcosgpu_init(int device) { return bcosgpu_init_ex(device, 0); }

int bcosgpu_init_ex(int device, int flags) { return init_device(device, flags); }

}  // extern "C"

namespace {
// selects `device` on the calling thread and builds its tables once
int init_device(int device, int flags) {
    int n = bcosgpu_device_count();
    if (n <= 0) return set_err(BCOSGPU_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return set_err(BCOSGPU_E_ARG, "device index out of range");
    HIP_OK(hipSetDevice(device));
    std::lock_guard<std::mutex> g(g_mu);
    if (g_ws.size() < static_cast<size_t>(n)) g_ws.resize(n, nullptr);
    if (!g_ws[device]) g_ws[device] = new Workspace();
    Workspace* w = g_ws[device];
    if (!w->ready) {
        hipDeviceProp_t prop;
        HIP_OK(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_err(BCOSGPU_E_NODEV, std::string("device is ") + prop.gcnArchName + ", built for gfx950");
        HIP_OK(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
        int rc = ecc_init_tables(device, (flags & BCOSGPU_INIT_SMALL_TABLES) != 0);
        if (rc) return set_err(rc, "ecc table setup failed");
        w->ready = true;
        if (device < 64) g_ready[device].store(true, std::memory_order_release);
    }
    return 0;
}
}  // namespace

extern "C" {

int bcosgpu_set_tx_kernel_policy(int split, int occupancy, int coop, int field) {
    set_tx_kernel_policy(split, occupancy, coop, field);
    return 0;
}

// ------------------------------------------------------------------ hashing
int bcosgpu_hash_batch_dev(int hasher, const uint8_t* d_data, const uint64_t* d_offsets, size_t n,
                           uint8_t* d_out32, void* stream) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (n && (!d_data || !d_offsets || !d_out32)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_hash_batch(hasher, d_data, d_offsets, n, d_out32, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "hash_batch launch") : 0;
}

int bcosgpu_hash_batch(int hasher, const uint8_t* data, const uint64_t* offsets, size_t n,
                       uint8_t* out32) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (n == 0) return 0;
    if (!data || !offsets || !out32) return set_err(BCOSGPU_E_ARG, "null pointer");
    const uint64_t base = offsets[0], bytes = offsets[n] - base;
    for (size_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 0xFFFFFFFFull)
            return set_err(BCOSGPU_E_ARG, "offsets must be non-decreasing and messages < 4 GiB");
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    HIP_OK(w->b[0].ensure(bytes + 8));
    HIP_OK(w->b[1].ensure((n + 1) * 8));
    HIP_OK(w->b[2].ensure(n * 32));
    std::vector<uint64_t> off(n + 1);
    for (size_t i = 0; i <= n; ++i) off[i] = offsets[i] - base;
    HIP_OK(hipMemcpyAsync(w->b[0].p, data + base, bytes, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[1].p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, w->stream));
    rc = launch_hash_batch(hasher, w->b[0].as<uint8_t>(), w->b[1].as<uint64_t>(), n, w->b[2].as<uint8_t>(), w->stream);
    if (rc) return hip_err(hipGetLastError(), "hash_batch launch");
    HIP_OK(hipMemcpyAsync(out32, w->b[2].p, n * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

int bcosgpu_keccak256_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
    return bcosgpu_hash_batch(BCOSGPU_KECCAK256, data, offsets, n, out32);
}
int bcosgpu_sm3_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
    return bcosgpu_hash_batch(BCOSGPU_SM3, data, offsets, n, out32);
}

// ------------------------------------------------------------------ Merkle
int bcosgpu_merkle_root_dev(int hasher, int width, const uint8_t* d_leaves32, size_t n,
                            uint8_t* d_tree, uint8_t* d_root32, void* stream) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (!d_leaves32 || !d_tree) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle(hasher, width, d_leaves32, n, d_tree, d_root32, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle launch") : 0;
}

uint64_t bcosgpu_merkle_bytes_size(uint64_t n, int width) {
    if (width < 2 || n == 0) return 0;
    return n == 1 ? 32 : 32 * merkle_size(n, width) - 28 * merkle_levels(n, width);
}

int bcosgpu_merkle_tree_bytes_dev(int width, const uint8_t* d_tree, size_t n, uint8_t* d_out, void* stream) {
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
    if (!d_tree || !d_out) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle_compact(d_tree, n, width, d_out, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle compact launch") : 0;
}

int bcosgpu_merkle_root(int hasher, int width, int variant, const uint8_t* leaves32, size_t n,
                        uint8_t* root32, uint8_t* levels) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (!root32 || (n && !leaves32)) return set_err(BCOSGPU_E_ARG, "null pointer");
    const bool bytes_layout = variant == BCOSGPU_MERKLE_NEW_BYTES;
    if (bytes_layout) variant = BCOSGPU_MERKLE_NEW;
    if (variant == BCOSGPU_MERKLE_NEW) {
        if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
        if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    } else if (variant != BCOSGPU_MERKLE_OLD) {
        return set_err(BCOSGPU_E_ARG, "bad variant");
    }
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    const uint64_t tree = variant == BCOSGPU_MERKLE_NEW ? bcosgpu_merkle_size(n, width) : merkle_size(n, 16) + 1;
    HIP_OK(w->b[0].ensure(n * 32 + 32));
    HIP_OK(w->b[1].ensure(tree * 32 + 32));
    HIP_OK(w->b[2].ensure(32));
    if (levels && bytes_layout) HIP_OK(w->b[3].ensure(tree * 32 + 32));
    if (n) HIP_OK(hipMemcpyAsync(w->b[0].p, leaves32, n * 32, hipMemcpyHostToDevice, w->stream));
    if (variant == BCOSGPU_MERKLE_NEW)
        rc = launch_merkle(hasher, width, w->b[0].as<uint8_t>(), n, w->b[1].as<uint8_t>(), w->b[2].as<uint8_t>(), w->stream);
    else
        rc = launch_merkle_old(hasher, w->b[0].as<uint8_t>(), n, w->b[1].as<uint8_t>(), w->b[2].as<uint8_t>(), w->stream);
    if (!rc && levels && bytes_layout)
        rc = launch_merkle_compact(w->b[1].as<uint8_t>(), n, width, w->b[3].as<uint8_t>(), w->stream);
    if (rc) return rc == BCOSGPU_E_ARG ? set_err(rc, "bad merkle arguments") : hip_err(hipGetLastError(), "merkle launch");
    HIP_OK(hipMemcpyAsync(root32, w->b[2].p, 32, hipMemcpyDeviceToHost, w->stream));
    if (levels && bytes_layout)
        HIP_OK(hipMemcpyAsync(levels, w->b[3].p, bcosgpu_merkle_bytes_size(n, width), hipMemcpyDeviceToHost, w->stream));
    else if (levels && variant == BCOSGPU_MERKLE_NEW)
        HIP_OK(hipMemcpyAsync(levels, w->b[1].p, tree * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

int bcosgpu_merkle_frontier_dev(int hasher, int width, const uint8_t* d_leaves32, size_t n, int levels,
                                uint8_t* d_work, uint8_t* d_frontier, void* stream) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
    if (width < 2 || width > 64 || levels < 1 || levels > 63) return set_err(BCOSGPU_E_ARG, "bad width/levels");
    if (!d_leaves32 || !d_work || !d_frontier) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle_levels(hasher, width, d_leaves32, n, levels, d_work, d_frontier, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle frontier launch") : 0;
}

uint64_t bcosgpu_merkle_roots_work_size(uint64_t total_leaves, size_t nblocks, int width) {
    if (width < 2 || width > 64) return 0;
    return merkle_roots_work_bytes(total_leaves, nblocks, width);
}

static int check_block_off(const uint64_t* block_off, size_t nblocks) {
    if (!block_off) return set_err(BCOSGPU_E_ARG, "null block offsets");
    for (size_t b = 0; b < nblocks; ++b)
        if (block_off[b + 1] < block_off[b] || block_off[b + 1] - block_off[b] > 0xFFFFFFFFull)
            return set_err(BCOSGPU_E_ARG, "block offsets must be non-decreasing, blocks < 2^32 leaves");
    return 0;
}

int bcosgpu_merkle_roots_batch_dev(int hasher, int width, const uint8_t* d_leaves32, const uint64_t* block_off,
                                   size_t nblocks, uint8_t* d_work, uint8_t* d_roots32, void* stream) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (nblocks == 0) return 0;
    if (int rc = check_block_off(block_off, nblocks)) return rc;
    if (!d_work || !d_roots32 || (block_off[nblocks] > block_off[0] && !d_leaves32))
        return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle_roots_batch(hasher, width, d_leaves32, block_off, nblocks, d_work, d_roots32,
                                       as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle roots launch") : 0;
}

int bcosgpu_merkle_roots_batch(int hasher, int width, const uint8_t* leaves32, const uint64_t* block_off,
                               size_t nblocks, uint8_t* roots32) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (nblocks == 0) return 0;
    if (int rc = check_block_off(block_off, nblocks)) return rc;
    const uint64_t total = block_off[nblocks] - block_off[0];
    if (!roots32 || (total && !leaves32)) return set_err(BCOSGPU_E_ARG, "null pointer");
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    HIP_OK(w->b[0].ensure(total * 32 + 32));
    HIP_OK(w->b[1].ensure(merkle_roots_work_bytes(total, nblocks, width)));
    HIP_OK(w->b[2].ensure(nblocks * 32));
    if (total) HIP_OK(hipMemcpyAsync(w->b[0].p, leaves32, total * 32, hipMemcpyHostToDevice, w->stream));
    rc = launch_merkle_roots_batch(hasher, width, w->b[0].as<uint8_t>(), block_off, nblocks, w->b[1].as<uint8_t>(),
                                   w->b[2].as<uint8_t>(), w->stream);
    if (rc) return hip_err(hipGetLastError(), "merkle roots launch");
    HIP_OK(hipMemcpyAsync(roots32, w->b[2].p, nblocks * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

// calculateReceiptRoot for many blocks (BlockImpl.h:156-183): the receipt preimages are packed
// (pack.cpp, TarsHashable.h:54-73) straight into pinned staging, one H2D, one hash launch, the dataHash
// short-circuits (TarsHashable.h:47-51) patched in, then the many-tree root kernel.
int bcosgpu_receipt_roots(int hasher, const bcosgpu_TransactionReceiptData* receipts, const uint64_t* block_off,
                          size_t nblocks, uint8_t* roots32, uint8_t* hashes32) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (nblocks == 0) return 0;
    if (int rc = check_block_off(block_off, nblocks)) return rc;
    if (block_off[0] != 0) return set_err(BCOSGPU_E_ARG, "block_off[0] must be 0");
    const uint64_t n = block_off[nblocks];
    if (!roots32 || (n && !receipts)) return set_err(BCOSGPU_E_ARG, "null pointer");
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    const uint64_t bytes = bcosgpu_receipt_preimage_size(receipts, n);
    bool patched = false;
    for (uint64_t i = 0; i < n && !patched; ++i) patched = receipts[i].data_hash_len != 0;
    HIP_OK(w->h[0].ensure(bytes + 8 * (n + 1) + 16));
    if (patched) HIP_OK(w->h[1].ensure(32 * n + 32));
    uint64_t* off = w->h[0].as<uint64_t>();
    uint8_t* pre = reinterpret_cast<uint8_t*>(off + n + 1);
    if (bcosgpu_pack_receipt_preimages(receipts, n, pre, bytes, off))
        return set_err(BCOSGPU_E_ARG, "bad receipt view (null field with a length, or a dataHash over 32 bytes)");
    HIP_OK(w->b[0].ensure(bytes + 8 * (n + 1) + 16));
    HIP_OK(w->b[1].ensure(32 * n + 32));
    HIP_OK(w->b[2].ensure(merkle_roots_work_bytes(n, nblocks, 2)));
    HIP_OK(w->b[3].ensure(nblocks * 32));
    uint8_t* d_hash = w->b[1].as<uint8_t>();
    if (n) {
        HIP_OK(hipMemcpyAsync(w->b[0].p, off, bytes + 8 * (n + 1), hipMemcpyHostToDevice, w->stream));
        const uint64_t* d_off = w->b[0].as<uint64_t>();
        if (launch_hash_batch(hasher, reinterpret_cast<const uint8_t*>(d_off + n + 1), d_off, n, d_hash, w->stream))
            return hip_err(hipGetLastError(), "receipt hash launch");
        if (patched) {  // the dataHash receipts: hashes round-trip through the host once
            uint8_t* h = w->h[1].as<uint8_t>();
            HIP_OK(hipMemcpyAsync(h, d_hash, 32 * n, hipMemcpyDeviceToHost, w->stream));
            HIP_OK(hipStreamSynchronize(w->stream));
            bcosgpu_apply_receipt_data_hashes(receipts, n, h);
            HIP_OK(hipMemcpyAsync(d_hash, h, 32 * n, hipMemcpyHostToDevice, w->stream));
        }
    }
    rc = launch_merkle_roots_batch(hasher, 2, d_hash, block_off, nblocks, w->b[2].as<uint8_t>(), w->b[3].as<uint8_t>(),
                                   w->stream);
    if (rc) return hip_err(hipGetLastError(), "merkle roots launch");
    HIP_OK(hipMemcpyAsync(roots32, w->b[3].p, nblocks * 32, hipMemcpyDeviceToHost, w->stream));
    if (hashes32 && n) HIP_OK(hipMemcpyAsync(hashes32, d_hash, 32 * n, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

// ------------------------------------------------------------------ Merkle proofs
uint64_t bcosgpu_merkle_proof_stride(uint64_t n, int width) {
    if (width < 2 || width > 64 || n == 0) return 0;
    return merkle_proof_stride(n, width);
}

int bcosgpu_merkle_proofs_dev(int width, const uint8_t* d_leaves32, size_t n, const uint8_t* d_tree,
                              const uint64_t* d_index, size_t m, uint8_t* d_proofs, uint32_t* d_proof_len, void* stream) {
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
    if (m && (!d_leaves32 || !d_tree || !d_index || !d_proofs || !d_proof_len)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle_proofs(width, d_leaves32, n, d_tree, d_index, m, d_proofs, d_proof_len, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle proofs launch") : 0;
}

int bcosgpu_merkle_proofs(int hasher, int width, const uint8_t* leaves32, size_t n, const uint64_t* index, size_t m,
                          uint8_t* proofs, uint32_t* proof_len) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (width < 2 || width > 64) return set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (n == 0) return set_err(BCOSGPU_E_EMPTY, "Empty input");
    if (m == 0) return 0;
    if (!leaves32 || !index || !proofs || !proof_len) return set_err(BCOSGPU_E_ARG, "null pointer");
    for (size_t q = 0; q < m; ++q)
        if (index[q] >= n) return set_err(BCOSGPU_E_ARG, "Out of range!");  // Merkle.h:124-127
    const uint64_t stride = merkle_proof_stride(n, width), tree = bcosgpu_merkle_size(n, width);
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    HIP_OK(w->b[0].ensure(n * 32));
    HIP_OK(w->b[1].ensure(tree * 32 + 32));
    HIP_OK(w->b[2].ensure(m * 8));
    HIP_OK(w->b[3].ensure(m * stride * 32));
    HIP_OK(w->b[4].ensure(m * 4));
    HIP_OK(hipMemcpyAsync(w->b[0].p, leaves32, n * 32, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[2].p, index, m * 8, hipMemcpyHostToDevice, w->stream));
    rc = launch_merkle(hasher, width, w->b[0].as<uint8_t>(), n, w->b[1].as<uint8_t>(), nullptr, w->stream);
    if (!rc)
        rc = launch_merkle_proofs(width, w->b[0].as<uint8_t>(), n, w->b[1].as<uint8_t>(), w->b[2].as<uint64_t>(), m,
                                  w->b[3].as<uint8_t>(), w->b[4].as<uint32_t>(), w->stream);
    if (rc) return hip_err(hipGetLastError(), "merkle proofs launch");
    HIP_OK(hipMemcpyAsync(proofs, w->b[3].p, m * stride * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipMemcpyAsync(proof_len, w->b[4].p, m * 4, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

int bcosgpu_merkle_verify_proofs_dev(int hasher, const uint8_t* d_proofs, uint64_t stride, const uint32_t* d_proof_len,
                                     const uint8_t* d_hashes32, const uint8_t* d_roots32, int per_proof_root, size_t m,
                                     uint8_t* d_ok, void* stream) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (stride == 0 || stride > 0xFFFFFFFFull) return set_err(BCOSGPU_E_ARG, "bad proof stride");
    if (m && (!d_proofs || !d_proof_len || !d_hashes32 || !d_roots32 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_merkle_verify(hasher, d_proofs, stride, d_proof_len, d_hashes32, d_roots32, per_proof_root ? 1 : 0, m,
                                  d_ok, as_stream(stream));
    return rc ? hip_err(hipGetLastError(), "merkle verify launch") : 0;
}

int bcosgpu_merkle_verify_proofs(int hasher, const uint8_t* proofs, uint64_t stride, const uint32_t* proof_len,
                                 const uint8_t* hashes32, const uint8_t* roots32, int per_proof_root, size_t m, uint8_t* ok) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return set_err(BCOSGPU_E_ARG, "bad hasher");
    if (stride == 0 || stride > 0xFFFFFFFFull) return set_err(BCOSGPU_E_ARG, "bad proof stride");
    if (m == 0) return 0;
    if (!proofs || !proof_len || !hashes32 || !roots32 || !ok) return set_err(BCOSGPU_E_ARG, "null pointer");
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    const size_t nroots = per_proof_root ? m : 1;
    HIP_OK(w->b[0].ensure(m * stride * 32));
    HIP_OK(w->b[1].ensure(m * 4));
    HIP_OK(w->b[2].ensure(m * 32));
    HIP_OK(w->b[3].ensure(nroots * 32));
    HIP_OK(w->b[4].ensure(m));
    HIP_OK(hipMemcpyAsync(w->b[0].p, proofs, m * stride * 32, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[1].p, proof_len, m * 4, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[2].p, hashes32, m * 32, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[3].p, roots32, nroots * 32, hipMemcpyHostToDevice, w->stream));
    rc = launch_merkle_verify(hasher, w->b[0].as<uint8_t>(), stride, w->b[1].as<uint32_t>(), w->b[2].as<uint8_t>(),
                              w->b[3].as<uint8_t>(), per_proof_root ? 1 : 0, m, w->b[4].as<uint8_t>(), w->stream);
    if (rc) return hip_err(hipGetLastError(), "merkle verify launch");
    HIP_OK(hipMemcpyAsync(ok, w->b[4].p, m, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

// ------------------------------------------------------------------ signatures
int bcosgpu_secp256k1_recover_batch_dev(const uint8_t* d_hash32, const uint8_t* d_sig65, size_t n,
                                        uint8_t* d_pub64, uint8_t* d_addr20, uint8_t* d_ok,
                                        void* stream) {
    if (n && (!d_hash32 || !d_sig65 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_secp256k1_recover(d_hash32, d_sig65, 65, n, d_pub64, d_addr20, d_ok, as_stream(stream));
    return rc ? set_err(rc, "secp256k1 recover launch failed") : 0;
}

int bcosgpu_secp256k1_recover_batch(const uint8_t* hash32, const uint8_t* sig65, size_t n,
                                    uint8_t* pub64, uint8_t* addr20, uint8_t* ok) {
    if (n == 0) return 0;
    if (!hash32 || !sig65 || !ok) return set_err(BCOSGPU_E_ARG, "null pointer");
    int dev = 0;
    if (int rc = calling_device(&dev)) return rc;
    SigJob job;
    job.kind = kSigJobRecoverK1;
    job.n = n;
    job.hash32 = hash32;
    job.sig = sig65;
    job.sig_stride = 65;
    job.out_pub64 = pub64;
    job.out_addr20 = addr20;
    job.out_ok = ok;
    return run_job(dev, job);
}

int bcosgpu_sm2_verify_batch_dev(const uint8_t* d_hash32, const uint8_t* d_sig128, size_t n,
                                 uint8_t* d_addr20, uint8_t* d_ok, void* stream) {
    if (n && (!d_hash32 || !d_sig128 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_sm2_verify(d_hash32, d_sig128, 128, n, d_addr20, d_ok, as_stream(stream));
    return rc ? set_err(rc, "sm2 verify launch failed") : 0;
}

int bcosgpu_sm2_verify_batch(const uint8_t* hash32, const uint8_t* sig128, size_t n,
                             uint8_t* addr20, uint8_t* ok) {
    if (n == 0) return 0;
    if (!hash32 || !sig128 || !ok) return set_err(BCOSGPU_E_ARG, "null pointer");
    int dev = 0;
    if (int rc = calling_device(&dev)) return rc;
    SigJob job;
    job.kind = kSigJobVerifySM2;
    job.n = n;
    job.hash32 = hash32;
    job.sig = sig128;
    job.sig_stride = 128;
    job.out_addr20 = addr20;
    job.out_ok = ok;
    return run_job(dev, job);
}

int bcosgpu_secp256k1_sign_batch_dev(const uint8_t* d_sk32, const uint8_t* d_hash32, size_t n,
                                     uint8_t* d_pub64, uint8_t* d_sig65, uint8_t* d_ok, void* stream) {
    if (n && (!d_sk32 || !d_hash32 || !d_sig65 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_secp256k1_sign(d_sk32, d_hash32, n, d_pub64, d_sig65, d_ok, as_stream(stream));
    return rc ? set_err(rc, "secp256k1 sign launch failed") : 0;
}

int bcosgpu_sm2_sign_batch_dev(const uint8_t* d_sk32, const uint8_t* d_hash32, size_t n,
                               uint8_t* d_sig128, uint8_t* d_ok, void* stream) {
    if (n && (!d_sk32 || !d_hash32 || !d_sig128 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_sm2_sign(d_sk32, d_hash32, n, d_sig128, d_ok, as_stream(stream));
    return rc ? set_err(rc, "sm2 sign launch failed") : 0;
}

// ------------------------------------------------------------------ verify with a known key, ecRecover
int bcosgpu_verify_batch_dev(int suite, const uint8_t* d_pub64, const uint8_t* d_hash32, const uint8_t* d_sig,
                             size_t sig_stride, size_t n, uint8_t* d_ok, void* stream) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (sig_stride < 64 || sig_stride > 0xFFFFFFFFull) return set_err(BCOSGPU_E_ARG, "signature stride must be >= 64");
    if (n && (!d_pub64 || !d_hash32 || !d_sig || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_sig_verify(suite, d_pub64, d_hash32, d_sig, static_cast<uint32_t>(sig_stride), n, d_ok,
                               as_stream(stream));
    return rc ? set_err(rc, "verify launch failed") : 0;
}

int bcosgpu_verify_batch(int suite, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig,
                         size_t sig_stride, size_t n, uint8_t* ok) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (sig_stride < 64 || sig_stride > 0xFFFFFFFFull) return set_err(BCOSGPU_E_ARG, "signature stride must be >= 64");
    if (n == 0) return 0;
    if (!pub64 || !hash32 || !sig || !ok) return set_err(BCOSGPU_E_ARG, "null pointer");
    int dev = 0;
    if (int rc = calling_device(&dev)) return rc;
    SigJob job;
    job.kind = suite == BCOSGPU_SUITE_SM2 ? kSigJobVerifySM2 : kSigJobVerifyK1;
    job.n = n;
    job.hash32 = hash32;
    job.sig = sig;
    job.sig_stride = sig_stride;
    job.pub64 = pub64;
    job.out_ok = ok;
    return run_job(dev, job);
}

// ------------------------------------------------------------------ registered keys (ecc_keyed.hip)
int bcosgpu_register_keys(int device, int suite, const uint8_t* pub64, size_t n, int32_t* slots) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (n && (!pub64 || !slots)) return set_err(BCOSGPU_E_ARG, "null pointer");
    if (int rc = ready_device(device)) return rc;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) {
        (void)hipGetLastError();
        prev = -1;
    }
    if (prev != device && hipSetDevice(device) != hipSuccess) return set_err(BCOSGPU_E_HIP, "hipSetDevice failed");
    bool all = false;
    const int rc = keyed_slots(suite, pub64, 64, n, slots, true, &all, nullptr);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (rc) return set_err(rc, "key table build failed");
    int cached = 0;
    for (size_t i = 0; i < n; ++i) cached += slots[i] >= 0;
    return cached;
}

int bcosgpu_verify_keyed_batch_dev(int suite, const int32_t* d_slots, const uint8_t* d_hash32, const uint8_t* d_sig,
                                   size_t sig_stride, size_t n, uint8_t* d_ok, void* stream) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (sig_stride < 64 || sig_stride > 0xFFFFFFFFull) return set_err(BCOSGPU_E_ARG, "signature stride must be >= 64");
    if (n && (!d_slots || !d_hash32 || !d_sig || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    const int rc = launch_sig_verify_keyed(suite, d_slots, d_hash32, d_sig, static_cast<uint32_t>(sig_stride), n, d_ok,
                                           nullptr, as_stream(stream));
    return rc ? set_err(rc, rc == BCOSGPU_E_ARG ? "no key registered on this device" : "keyed verify launch failed") : 0;
}

int bcosgpu_key_cache_info(int device, int suite, int64_t* out5) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (!out5) return set_err(BCOSGPU_E_ARG, "null pointer");
    const int rc = keyed_cache_info(device, suite, out5);
    return rc ? set_err(rc, "bad device") : 0;
}

int bcosgpu_clear_keys(int device, int suite) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    const int rc = keyed_clear(device, suite);
    return rc ? set_err(rc, "clearing the key cache failed") : 0;
}

int bcosgpu_ecrecover_batch_dev(const uint8_t* d_in128, size_t n, uint8_t* d_out32, uint8_t* d_ok, void* stream) {
    if (n && (!d_in128 || !d_out32 || !d_ok)) return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_ecrecover(d_in128, n, d_out32, d_ok, as_stream(stream));
    return rc ? set_err(rc, "ecrecover launch failed") : 0;
}

int bcosgpu_ecrecover_batch(const uint8_t* in128, size_t n, uint8_t* out32, uint8_t* ok) {
    if (n == 0) return 0;
    if (!in128 || !out32 || !ok) return set_err(BCOSGPU_E_ARG, "null pointer");
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    HIP_OK(w->b[0].ensure(n * 128));
    HIP_OK(w->b[1].ensure(n * 32));
    HIP_OK(w->b[2].ensure(n));
    HIP_OK(hipMemcpyAsync(w->b[0].p, in128, n * 128, hipMemcpyHostToDevice, w->stream));
    rc = launch_ecrecover(w->b[0].as<uint8_t>(), n, w->b[1].as<uint8_t>(), w->b[2].as<uint8_t>(), w->stream);
    if (rc) return set_err(rc, "ecrecover launch failed");
    HIP_OK(hipMemcpyAsync(out32, w->b[1].p, n * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipMemcpyAsync(ok, w->b[2].p, n, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

// ------------------------------------------------------------------ whole-tx admission
int bcosgpu_tx_verify_batch_dev(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off,
                                const uint8_t* d_sig, const uint64_t* d_sig_off, size_t n,
                                uint8_t* d_txhash32, uint8_t* d_sender20, uint8_t* d_status,
                                void* stream) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (n && (!d_pre || !d_pre_off || !d_sig || !d_sig_off || !d_txhash32 || !d_sender20 || !d_status))
        return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_tx_verify(suite, d_pre, d_pre_off, d_sig, d_sig_off, n, d_txhash32, d_sender20, d_status,
                              as_stream(stream));
    return rc ? set_err(rc, "tx verify launch failed") : 0;
}

// The batch site TransactionSync::importDownloadedTxs (TransactionSync.cpp:516-548) holds host memory:
// the chunked copy / compute pipeline of txpipe.hip on a pipeline of the calling thread's device (its own
// streams and buffers: concurrent callers overlap).
int bcosgpu_tx_verify_batch(int suite, const uint8_t* pre, const uint64_t* pre_off,
                            const uint8_t* sig, const uint64_t* sig_off, size_t n,
                            uint8_t* txhash32, uint8_t* sender20, uint8_t* status) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (n == 0) return 0;
    if (!pre || !pre_off || !sig || !sig_off || !txhash32 || !sender20 || !status)
        return set_err(BCOSGPU_E_ARG, "null pointer");
    int dev = 0;  // (the offsets are checked by the pipeline, chunk by chunk)
    if (int rc = calling_device(&dev)) return rc;
    TxPipe* p = tx_pipe_acquire(dev);
    if (!p) return hip_err(hipGetLastError(), "tx pipeline setup");
    HostTxRange t;
    t.suite = suite;
    t.pre = pre;
    t.pre_off = pre_off;
    t.sig = sig;
    t.sig_off = sig_off;
    t.lo = 0;
    t.hi = n;
    t.txhash32 = txhash32;
    t.sender20 = sender20;
    t.status = status;
    std::string msg;
    const int rc = tx_pipeline(*p, t, nullptr, msg);
    tx_pipe_release(p);
    return rc ? set_err(rc, msg) : 0;
}

// ------------------------------------------------------------------ Tars-encoded transactions
uint64_t bcosgpu_tars_decode_work_size(size_t n) { return tars_decode_work_bytes(n); }

int bcosgpu_tars_tx_decode_dev(const uint8_t* d_enc, const uint64_t* d_enc_off, size_t n, uint8_t* d_pre,
                               uint64_t* d_pre_off, uint8_t* d_sig, uint64_t* d_sig_off, uint8_t* d_dec_status,
                               void* d_work, uint64_t work_bytes, void* stream) {
    if (n == 0) return 0;
    if (!d_enc || !d_enc_off || !d_pre || !d_pre_off || !d_sig || !d_sig_off || !d_work)
        return set_err(BCOSGPU_E_ARG, "null pointer");
    int rc = launch_tars_tx_decode(d_enc, d_enc_off, n, d_pre, d_pre_off, d_sig, d_sig_off, d_dec_status, d_work,
                                   work_bytes, as_stream(stream));
    if (rc == BCOSGPU_E_ARG) return set_err(rc, "work buffer too small or batch too large");
    return rc ? hip_err(hipGetLastError(), "tars decode launch") : 0;
}

int bcosgpu_tars_tx_verify_batch_dev(int suite, const uint8_t* d_enc, const uint64_t* d_enc_off, size_t n,
                                     int check_sig, int check_hash, uint8_t* d_pre, uint64_t* d_pre_off, uint8_t* d_sig,
                                     uint64_t* d_sig_off, void* d_work, uint64_t work_bytes, uint8_t* d_txhash32,
                                     uint8_t* d_sender20, uint8_t* d_status, void* stream) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (n == 0) return 0;
    if (!d_enc || !d_enc_off || !d_pre || !d_pre_off || !d_sig || !d_sig_off || !d_work || !d_txhash32 ||
        !d_sender20 || !d_status)
        return set_err(BCOSGPU_E_ARG, "null pointer");
    hipStream_t st = as_stream(stream);
    int rc = launch_tars_tx_decode(d_enc, d_enc_off, n, d_pre, d_pre_off, d_sig, d_sig_off, nullptr, d_work,
                                   work_bytes, st);
    if (rc == BCOSGPU_E_ARG) return set_err(rc, "work buffer too small or batch too large");
    if (!rc && check_sig) {
        rc = launch_tx_verify(suite, d_pre, d_pre_off, d_sig, d_sig_off, n, d_txhash32, d_sender20, d_status, st);
    } else if (!rc) {  // checkSig = false: decode + hash only (TransactionFactoryImpl.h:52-60)
        rc = launch_hash_batch(suite == BCOSGPU_SUITE_SM2 ? BCOSGPU_SM3 : BCOSGPU_KECCAK256, d_pre, d_pre_off, n,
                               d_txhash32, st);
        if (!rc && (hipMemsetAsync(d_sender20, 0, 20 * n, st) != hipSuccess ||
                    hipMemsetAsync(d_status, 0, n, st) != hipSuccess))
            rc = BCOSGPU_E_HIP;
    }
    if (!rc) rc = launch_tars_finish(d_enc, d_work, nullptr, d_txhash32, d_status, n, check_hash, st);
    return rc ? hip_err(hipGetLastError(), "tars tx verify launch") : 0;
}

int bcosgpu_tars_tx_verify_batch(int suite, const uint8_t* enc, const uint64_t* enc_off, size_t n, int check_sig,
                                 int check_hash, uint8_t* txhash32, uint8_t* sender20, uint8_t* status) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return set_err(BCOSGPU_E_ARG, "bad suite");
    if (n == 0) return 0;
    if (!enc || !enc_off || !txhash32 || !sender20 || !status) return set_err(BCOSGPU_E_ARG, "null pointer");
    for (size_t i = 0; i < n; ++i)
        if (enc_off[i + 1] < enc_off[i]) return set_err(BCOSGPU_E_ARG, "offsets must be non-decreasing");
    const uint64_t base = enc_off[0], bytes = enc_off[n] - base;
    Workspace* w;
    int rc = get_ws(&w);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(w->mu);
    const uint64_t work = tars_decode_work_bytes(n);
    HIP_OK(w->b[0].ensure(bytes + 8));
    HIP_OK(w->b[1].ensure((n + 1) * 8));
    HIP_OK(w->b[2].ensure(bytes + 12 * n + 8));  // preimages
    HIP_OK(w->b[3].ensure(2 * (n + 1) * 8));     // preimage + signature offsets
    HIP_OK(w->b[4].ensure(bytes + 8));           // signatures
    HIP_OK(w->b[5].ensure(n * 53));              // txhash, sender, status
    HIP_OK(w->b[6].ensure(work));
    std::vector<uint64_t> off(n + 1);
    for (size_t i = 0; i <= n; ++i) off[i] = enc_off[i] - base;
    HIP_OK(hipMemcpyAsync(w->b[0].p, enc + base, bytes, hipMemcpyHostToDevice, w->stream));
    HIP_OK(hipMemcpyAsync(w->b[1].p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, w->stream));
    uint64_t* pre_off = w->b[3].as<uint64_t>();
    uint8_t* out = w->b[5].as<uint8_t>();
    rc = bcosgpu_tars_tx_verify_batch_dev(suite, w->b[0].as<uint8_t>(), w->b[1].as<uint64_t>(), n, check_sig,
                                          check_hash,
                                          w->b[2].as<uint8_t>(), pre_off, w->b[4].as<uint8_t>(), pre_off + (n + 1),
                                          w->b[6].p, work, out, out + 32 * n, out + 52 * n, w->stream);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(txhash32, out, n * 32, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipMemcpyAsync(sender20, out + 32 * n, n * 20, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipMemcpyAsync(status, out + 52 * n, n, hipMemcpyDeviceToHost, w->stream));
    HIP_OK(hipStreamSynchronize(w->stream));
    return 0;
}

// ------------------------------------------------------------------ single calls (coalesced)
int bcosgpu_secp256k1_recover(int device, const uint8_t* hash32, const uint8_t* sig, size_t sig_len, uint8_t* pub64) {
    if (!hash32 || !sig || !pub64) return set_err(BCOSGPU_E_ARG, "null pointer");
    if (int rc = ready_device(device)) return rc;
    if (sig_len != 65) {  // SECP256K1_SIGNATURE_LEN (Secp256k1Crypto.h:29): InvalidSignature
        std::memset(pub64, 0, 64);
        return 0;
    }
    uint8_t ok = 0;
    SigJob job;
    job.kind = kSigJobRecoverK1;
    job.n = 1;
    job.hash32 = hash32;
    job.sig = sig;
    job.sig_stride = 65;
    job.out_pub64 = pub64;
    job.out_ok = &ok;
    if (int rc = run_job(device, job)) return rc;
    return ok ? 1 : 0;
}

int bcosgpu_secp256k1_verify(int device, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig,
                             size_t sig_len) {
    if (!pub64 || !hash32 || !sig) return set_err(BCOSGPU_E_ARG, "null pointer");
    if (int rc = ready_device(device)) return rc;
    if (sig_len < 64) return 0;
    uint8_t ok = 0;
    SigJob job;
    job.kind = kSigJobVerifyK1;
    job.n = 1;
    job.hash32 = hash32;
    job.sig = sig;
    job.sig_stride = 64;
    job.pub64 = pub64;
    job.out_ok = &ok;
    if (int rc = run_job(device, job)) return rc;
    return ok ? 1 : 0;
}

int bcosgpu_sm2_verify(int device, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig64) {
    if (!pub64 || !hash32 || !sig64) return set_err(BCOSGPU_E_ARG, "null pointer");
    if (int rc = ready_device(device)) return rc;
    uint8_t ok = 0;
    SigJob job;
    job.kind = kSigJobVerifySM2;
    job.n = 1;
    job.hash32 = hash32;
    job.sig = sig64;
    job.sig_stride = 64;
    job.pub64 = pub64;
    job.out_ok = &ok;
    if (int rc = run_job(device, job)) return rc;
    return ok ? 1 : 0;
}

int bcosgpu_coalesce_stats(int device, uint64_t* out10, int reset) {
    if (!out10) return set_err(BCOSGPU_E_ARG, "null pointer");
    const int rc = coalesce_stats(device, out10, 10, reset);
    return rc ? set_err(rc, "bad device") : 0;
}

// ------------------------------------------------------------------ wedpr-ABI shims
// On the calling thread's current device.  0 = WEDPR_SUCCESS, -1 = WEDPR_ERROR (invalid input or
// signature), BCOSGPU_WEDPR_ENGINE_ERROR = the engine failed (no device, HIP error): the message is in
// bcosgpu_last_error().
static int shim_device() {
    int dev = 0;
    return current_device(&dev) ? -1 : dev;
}

int8_t bcosgpu_wedpr_secp256k1_recover_public_key(const bcosgpu_CInputBuffer* hash,
                                                   const bcosgpu_CInputBuffer* sig,
                                                   bcosgpu_COutputBuffer* pub) {
    if (!hash || !sig || !pub || hash->len != 32 || pub->len < 64) return -1;
    const int dev = shim_device();
    if (dev < 0) return BCOSGPU_WEDPR_ENGINE_ERROR;
    const int rc = bcosgpu_secp256k1_recover(dev, reinterpret_cast<const uint8_t*>(hash->data),
                                             reinterpret_cast<const uint8_t*>(sig->data), sig->len,
                                             reinterpret_cast<uint8_t*>(pub->data));
    return rc < 0 ? BCOSGPU_WEDPR_ENGINE_ERROR : rc == 1 ? 0 : -1;
}

int8_t bcosgpu_wedpr_sm2_verify(const bcosgpu_CInputBuffer* pub, const bcosgpu_CInputBuffer* hash,
                                 const bcosgpu_CInputBuffer* sig) {
    if (!pub || !hash || !sig || hash->len != 32 || sig->len != 64 || pub->len != 64) return -1;
    const int dev = shim_device();
    if (dev < 0) return BCOSGPU_WEDPR_ENGINE_ERROR;
    const int rc = bcosgpu_sm2_verify(dev, reinterpret_cast<const uint8_t*>(pub->data),
                                      reinterpret_cast<const uint8_t*>(hash->data),
                                      reinterpret_cast<const uint8_t*>(sig->data));
    return rc < 0 ? BCOSGPU_WEDPR_ENGINE_ERROR : rc == 1 ? 0 : -1;
}

int8_t bcosgpu_wedpr_secp256k1_verify(const bcosgpu_CInputBuffer* pub, const bcosgpu_CInputBuffer* hash,
                                      const bcosgpu_CInputBuffer* sig) {
    if (!pub || !hash || !sig || hash->len != 32 || pub->len != 64 || sig->len < 64) return -1;
    const int dev = shim_device();
    if (dev < 0) return BCOSGPU_WEDPR_ENGINE_ERROR;
    const int rc = bcosgpu_secp256k1_verify(dev, reinterpret_cast<const uint8_t*>(pub->data),
                                            reinterpret_cast<const uint8_t*>(hash->data),
                                            reinterpret_cast<const uint8_t*>(sig->data), sig->len);
    return rc < 0 ? BCOSGPU_WEDPR_ENGINE_ERROR : rc == 1 ? 0 : -1;
}

}  // extern "C"
