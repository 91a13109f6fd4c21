// multi.hip -- the device-set entry points (include/bcos_gpu.h "device sets"): one process drives every
// GPU of its node through the C ABI it links.  A FISCO node is a single process with one CryptoSuite
// (libinitializer/ProtocolInitializer.cpp:102-124) and in-process batch sites (TransactionSync.cpp:516-548,
// BlockImpl.h:111-154), so the multi-GPU split of SURVEY 8(e) has to live behind the ABI, not in a
// process-per-GPU launcher.
//
//  - A batch is split by index into one contiguous shard per entry of the device list; shard k runs on
//    devices[k] from its own host thread, on its own stream and buffers (a ShardCtx per (device, k-th
//    occurrence of that device in the list), so {0, 0} is two shards on one GPU on distinct streams).
//  - Signature batches: each shard is a coalesced job on its device (coalesce.hip), exactly what the
//    single-device host calls run.
//  - Block check / Merkle root: shard starts are multiples of width^L (Merkle<H, width> groups every
//    level from index 0, Merkle.h:243-261), so shard k's level-L nodes ARE the reference tree's level-L
//    nodes for its range; each GPU reduces its shard to them (launch_merkle_levels), devices[0] gathers
//    the frontiers (a few KB) with peer copies over xGMI and runs the top levels.  Bit-identical to the
//    single-device root for every n.
#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>
#include <cstdlib>
#include <cstring>
#include "engine.h"

using namespace bcosgpu;

namespace {

struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
        const hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// a shard's stream and grow-only device buffers; its mutex is held by the call that uses it
struct ShardCtx {
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    Buf b[10];
};

std::mutex g_mmu;
std::map<std::pair<int, int>, ShardCtx*> g_ctx;  // never freed: no teardown races with the HIP runtime

// slot -1 is the gather context of devices[0]
ShardCtx* shard_ctx(int device, int slot) {
    std::lock_guard<std::mutex> g(g_mmu);
    ShardCtx*& c = g_ctx[{device, slot}];
    if (!c) {
        c = new ShardCtx();
        c->device = device;
    }
    return c;
}

struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

std::string hip_msg(hipError_t e, const char* what) { return std::string(what) + ": " + hipGetErrorString(e); }

#define SHARD_HIP(call)                                  \
    do {                                                 \
        const hipError_t e_ = (call);                    \
        if (e_ != hipSuccess) {                          \
            msg = hip_msg(e_, #call);                    \
            return BCOSGPU_E_HIP;                        \
        }                                                \
    } while (0)

int check_set(const int* devices, int ndev) {
    if (!devices || ndev < 1 || ndev > 64) return api_set_err(BCOSGPU_E_ARG, "device list: 1 to 64 entries");
    for (int k = 0; k < ndev; ++k)
        if (int rc = api_ready_device(devices[k])) return rc;
    return 0;
}

// shard k's context: devices[k], numbered by its occurrences among devices[0..k)
std::vector<ShardCtx*> contexts(const int* devices, int ndev) {
    std::vector<ShardCtx*> out(ndev);
    for (int k = 0; k < ndev; ++k) {
        int occ = 0;
        for (int j = 0; j < k; ++j) occ += devices[j] == devices[k];
        out[k] = shard_ctx(devices[k], occ);
    }
    return out;
}

// lock every context a call uses (sorted, so concurrent calls cannot deadlock)
std::vector<std::unique_lock<std::mutex>> lock_all(std::vector<ShardCtx*> cs) {
    std::sort(cs.begin(), cs.end());
    cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
    std::vector<std::unique_lock<std::mutex>> locks;
    for (ShardCtx* c : cs) locks.emplace_back(c->mu);
    return locks;
}

// f(k, msg) for every shard, shards 1.. on their own host threads; the first failing shard's code,
// with its message set on the calling thread
template <class F>
int run_shards(int ndev, F&& f) {
    std::vector<int> rc(ndev, 0);
    std::vector<std::string> msg(ndev);
    auto one = [&](int k) {
        try {
            rc[k] = f(k, msg[k]);
        } catch (const std::exception& e) {
            rc[k] = BCOSGPU_E_HIP;
            msg[k] = std::string("shard failed on the host: ") + e.what();
        }
    };
    std::vector<std::thread> th;
    for (int k = 1; k < ndev; ++k) {
        try {
            th.emplace_back(one, k);
        } catch (const std::exception&) {
            one(k);  // no thread: run the shard here
        }
    }
    one(0);
    for (auto& t : th) t.join();
    for (int k = 0; k < ndev; ++k)
        if (rc[k]) return api_set_err(rc[k], msg[k]);
    return 0;
}

// contiguous shards [lo, hi); with width >= 2 every lo is a multiple of width^L, L chosen so the gathered
// frontier stays small (<= ~64 nodes per shard) while the tree still has more than L levels
// (bcos_gpu/parallel.py choose_levels / shard_plan, the same rule)
struct Plan {
    std::vector<uint64_t> lo, hi;
    int levels = 0;
    uint64_t blk = 1;
    uint64_t count(int k) const { return hi[k] > lo[k] ? (hi[k] - lo[k] + blk - 1) / blk : 0; }
};
Plan make_plan(uint64_t n, int ndev, int width) {
    Plan p;
    if (width >= 2) {
        uint64_t b = 1;
        while (true) {
            const uint64_t nb = b * static_cast<uint64_t>(width);
            if (static_cast<uint64_t>(ndev) * 64u * nb > n || (n + nb - 1) / nb < 2) break;
            b = nb;
            ++p.levels;
        }
        p.blk = b;
    }
    const uint64_t per = (n + static_cast<uint64_t>(ndev) * p.blk - 1) / (static_cast<uint64_t>(ndev) * p.blk) * p.blk;
    p.lo.resize(ndev);
    p.hi.resize(ndev);
    for (int k = 0; k < ndev; ++k) {
        p.lo[k] = std::min<uint64_t>(k * per, n);
        p.hi[k] = std::min<uint64_t>((k + 1) * per, n);
    }
    return p;
}

std::mutex g_peer_mu;
std::vector<std::pair<int, int>> g_peer_done;

// BCOSGPU_MULTI_PEER=1 (read at each call; a test hook for one-GPU boxes): shards on devices[0] itself
// also take the cross-device branches -- enable_peers' probe and the hipMemcpyPeerAsync gather (a peer
// copy whose source and destination device are the same is legal) -- so a one-GPU run executes the code
// a multi-GPU node runs
bool force_peer() {
    const char* v = std::getenv("BCOSGPU_MULTI_PEER");
    return v && v[0] == '1';
}

// devices[0] reads the other devices' frontiers directly when the platform allows it (xGMI peer access);
// otherwise hipMemcpyPeerAsync stages through the host
void enable_peers(const int* devices, int ndev) {
    const bool force = force_peer();
    std::lock_guard<std::mutex> g(g_peer_mu);
    for (int k = 1; k < ndev; ++k) {
        const std::pair<int, int> pr{devices[0], devices[k]};
        if ((pr.first == pr.second && !force) ||
            std::find(g_peer_done.begin(), g_peer_done.end(), pr) != g_peer_done.end())
            continue;
        g_peer_done.push_back(pr);
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, pr.first, pr.second) == hipSuccess && can && pr.first != pr.second) {
            DeviceGuard dg(pr.first);
            (void)hipDeviceEnablePeerAccess(pr.second, 0);
        }
        (void)hipGetLastError();
    }
}

hipError_t ensure_stream(ShardCtx* c) {
    if (c->stream) return hipSuccess;
    return hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
}

// the top of the tree on devices[0]: gather the shards' level-L nodes (frontier[k], count(k) nodes on
// devices[k]) into one vector and run Merkle<H, width> over it
int gather_root(const int* devices, int ndev, const Plan& p, const std::vector<const uint8_t*>& frontier, int hasher,
                int width, ShardCtx* r, uint8_t* root32) {
    std::string msg;
    const int rc = [&]() -> int {
        DeviceGuard dg(r->device);
        SHARD_HIP(dg.err);
        SHARD_HIP(ensure_stream(r));
        uint64_t total = 0;
        for (int k = 0; k < ndev; ++k) total += p.count(k);
        SHARD_HIP(r->b[0].ensure(total * 32));
        SHARD_HIP(r->b[1].ensure((merkle_size(total, width) + 1) * 32));
        SHARD_HIP(r->b[2].ensure(32));
        const bool peer_all = force_peer();
        uint64_t at = 0;
        for (int k = 0; k < ndev; ++k) {
            const uint64_t m = p.count(k);
            if (!m) continue;
            uint8_t* dst = r->b[0].as<uint8_t>() + 32 * at;
            if (devices[k] == r->device && !peer_all)
                SHARD_HIP(hipMemcpyAsync(dst, frontier[k], 32 * m, hipMemcpyDeviceToDevice, r->stream));
            else
                SHARD_HIP(hipMemcpyPeerAsync(dst, r->device, frontier[k], devices[k], 32 * m, r->stream));
            at += m;
        }
        const int lrc = launch_merkle(hasher, width, r->b[0].as<uint8_t>(), total, r->b[1].as<uint8_t>(),
                                      r->b[2].as<uint8_t>(), r->stream);
        if (lrc) {
            msg = hip_msg(hipGetLastError(), "merkle top levels launch");
            return lrc;
        }
        SHARD_HIP(hipMemcpyAsync(root32, r->b[2].p, 32, hipMemcpyDeviceToHost, r->stream));
        SHARD_HIP(hipStreamSynchronize(r->stream));
        return 0;
    }();
    return rc ? api_set_err(rc, msg) : 0;
}

int sig_multi(const int* devices, int ndev, int kind, size_t n, const uint8_t* hash32, const uint8_t* sig,
              size_t sig_stride, const uint8_t* pub64, uint8_t* out_pub64, uint8_t* out_addr20, uint8_t* ok) {
    if (int rc = check_set(devices, ndev)) return rc;
    const Plan p = make_plan(n, ndev, 0);
    return run_shards(ndev, [&](int k, std::string& msg) -> int {
        const uint64_t lo = p.lo[k], m = p.hi[k] - p.lo[k];
        if (!m) return 0;
        SigJob job;
        job.kind = kind;
        job.n = m;
        job.hash32 = hash32 + 32 * lo;
        job.sig = sig + sig_stride * lo;
        job.sig_stride = sig_stride;
        job.pub64 = pub64 ? pub64 + 64 * lo : nullptr;
        job.out_pub64 = out_pub64 ? out_pub64 + 64 * lo : nullptr;
        job.out_addr20 = out_addr20 ? out_addr20 + 20 * lo : nullptr;
        job.out_ok = ok + lo;
        const int rc = coalesced_run(devices[k], job);
        if (rc) msg = job.err;
        return rc;
    });
}

// shards' pipelines (txpipe.hip) from each device's pool, returned when the call ends
struct Pipes {
    std::vector<TxPipe*> p;
    ~Pipes() {
        for (TxPipe* x : p) tx_pipe_release(x);
    }
    int acquire(const int* devices, int ndev) {
        p.assign(ndev, nullptr);
        for (int k = 0; k < ndev; ++k) {
            p[k] = tx_pipe_acquire(devices[k]);
            if (!p[k]) return api_set_err(BCOSGPU_E_HIP, "tx pipeline setup on a device of the set failed");
        }
        return 0;
    }
};

// shards with work on shard k's device, k included (its pipeline's chunking: txpipe.hip)
int shards_on_device(const int* devices, int ndev, int k, const std::function<bool(int)>& has_work) {
    int n = 1;
    for (int j = 0; j < ndev; ++j)
        if (j != k && devices[j] == devices[k] && has_work(j)) ++n;
    return n;
}

HostTxRange host_range(int suite, const uint8_t* pre, const uint64_t* pre_off, const uint8_t* sig,
                       const uint64_t* sig_off, uint64_t lo, uint64_t hi, uint8_t* txhash32, uint8_t* sender20,
                       uint8_t* status) {
    HostTxRange t;
    t.suite = suite;
    t.pre = pre;
    t.pre_off = pre_off;
    t.sig = sig;
    t.sig_off = sig_off;
    t.lo = lo;
    t.hi = hi;
    t.txhash32 = txhash32;
    t.sender20 = sender20;
    t.status = status;
    return t;
}

int tx_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off, const uint8_t* sig,
             const uint64_t* sig_off, size_t n, int width, uint8_t* txhash32, uint8_t* sender20, uint8_t* status,
             uint8_t* root32) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return api_set_err(BCOSGPU_E_ARG, "bad suite");
    if (root32 && (width < 2 || width > 64)) return api_set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (n == 0) {  // BlockImpl.h:114-119: a block without transactions has the zero root
        if (root32) std::memset(root32, 0, 32);
        return check_set(devices, ndev);
    }
    if (!pre || !pre_off || !sig || !sig_off || !txhash32 || !sender20 || !status)
        return api_set_err(BCOSGPU_E_ARG, "null pointer");
    if (pre_off[n] < pre_off[0] || sig_off[n] < sig_off[0])
        return api_set_err(BCOSGPU_E_ARG, "offsets must be non-decreasing");  // (each shard's pipeline checks the rest)
    if (int rc = check_set(devices, ndev)) return rc;
    if (root32) enable_peers(devices, ndev);
    const int hasher = suite == BCOSGPU_SUITE_SM2 ? BCOSGPU_SM3 : BCOSGPU_KECCAK256;
    const Plan p = make_plan(n, ndev, root32 ? width : 0);
    Pipes pipes;
    if (int rc = pipes.acquire(devices, ndev)) return rc;
    ShardCtx* top = root32 ? shard_ctx(devices[0], -1) : nullptr;
    std::unique_lock<std::mutex> top_lock;
    if (top) top_lock = std::unique_lock<std::mutex>(top->mu);
    std::vector<const uint8_t*> frontier(ndev, nullptr);
    int rc = run_shards(ndev, [&](int k, std::string& msg) -> int {
        const uint64_t lo = p.lo[k], hi = p.hi[k], m = hi - lo;
        if (!m) return 0;
        TxPipe& c = *pipes.p[k];
        DeviceGuard dg(c.device);
        SHARD_HIP(dg.err);
        // the shard's level-L frontier (or its hashes, L = 0), queued behind the last chunk's kernel
        PipeTail tail = [&](TxPipe& q, const uint8_t* d_hash, std::string& m2) -> int {
            if (!root32) return 0;
            if (p.levels == 0) {
                frontier[k] = d_hash;
                return 0;
            }
            if (q.b[5].ensure(64 * ((m + width - 1) / width)) != hipSuccess || q.b[6].ensure(32 * p.count(k)) != hipSuccess) {
                m2 = "frontier buffers: out of device memory";
                return BCOSGPU_E_HIP;
            }
            const int lrc = launch_merkle_levels(hasher, width, d_hash, m, p.levels, q.b[5].as<uint8_t>(),
                                                 q.b[6].as<uint8_t>(), q.compute);
            if (lrc) m2 = hip_msg(hipGetLastError(), "merkle frontier launch");
            frontier[k] = q.b[6].as<uint8_t>();
            return lrc;
        };
        HostTxRange r = host_range(suite, pre, pre_off, sig, sig_off, lo, hi, txhash32, sender20, status);
        r.share = shards_on_device(devices, ndev, k, [&](int j) { return p.hi[j] > p.lo[j]; });
        return tx_pipeline(c, r, tail, msg);
    });
    if (rc || !root32) return rc;
    return gather_root(devices, ndev, p, frontier, hasher, width, top, root32);
}

// Many blocks at once over the device set (a sync catch-up or a replay: configs[4]): whole blocks per
// device, contiguous ranges balanced by tx count; each device verifies its txs through the chunked
// pipeline and computes its blocks' roots with the many-tree level kernel (launch_merkle_roots_batch)
// behind the last chunk; no exchange.
int blocks_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off, const uint8_t* sig,
                 const uint64_t* sig_off, const uint64_t* block_off, size_t nblocks, int width, uint8_t* txhash32,
                 uint8_t* sender20, uint8_t* status, uint8_t* roots32) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return api_set_err(BCOSGPU_E_ARG, "bad suite");
    if (width < 2 || width > 64) return api_set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (nblocks == 0) return check_set(devices, ndev);
    if (!block_off || !roots32) return api_set_err(BCOSGPU_E_ARG, "null pointer");
    if (block_off[0] != 0) return api_set_err(BCOSGPU_E_ARG, "block_off[0] must be 0");
    for (size_t b = 0; b < nblocks; ++b)
        if (block_off[b + 1] < block_off[b] || block_off[b + 1] - block_off[b] > 0xFFFFFFFFull)
            return api_set_err(BCOSGPU_E_ARG, "block offsets must be non-decreasing");
    const uint64_t n = block_off[nblocks];
    if (n && (!pre || !pre_off || !sig || !sig_off || !txhash32 || !sender20 || !status))
        return api_set_err(BCOSGPU_E_ARG, "null pointer");
    if (n && (pre_off[n] < pre_off[0] || sig_off[n] < sig_off[0]))
        return api_set_err(BCOSGPU_E_ARG, "offsets must be non-decreasing");  // (each shard's pipeline checks the rest)
    if (int rc = check_set(devices, ndev)) return rc;
    const int hasher = suite == BCOSGPU_SUITE_SM2 ? BCOSGPU_SM3 : BCOSGPU_KECCAK256;
    // block ranges [bl[k], bl[k + 1]): device k's share ends at the first block boundary past (k + 1) n / ndev
    std::vector<size_t> bl(ndev + 1, nblocks);
    bl[0] = 0;
    for (int k = 1; k < ndev; ++k) {
        const uint64_t want = n * static_cast<uint64_t>(k) / static_cast<uint64_t>(ndev);
        size_t b = bl[k - 1];
        while (b < nblocks && block_off[b] < want) ++b;
        bl[k] = b;
    }
    Pipes pipes;
    if (int rc = pipes.acquire(devices, ndev)) return rc;
    return run_shards(ndev, [&](int k, std::string& msg) -> int {
        const size_t b0 = bl[k], b1 = bl[k + 1], nb = b1 - b0;
        if (nb == 0) return 0;
        const uint64_t lo = block_off[b0], hi = block_off[b1], m = hi - lo;
        if (m == 0) {  // only empty blocks: zero roots (BlockImpl.h:114-119)
            std::memset(roots32 + 32 * b0, 0, 32 * nb);
            return 0;
        }
        TxPipe& c = *pipes.p[k];
        DeviceGuard dg(c.device);
        SHARD_HIP(dg.err);
        std::vector<uint64_t> boff(nb + 1);
        for (size_t b = 0; b <= nb; ++b) boff[b] = block_off[b0 + b] - lo;
        SHARD_HIP(c.b[5].ensure(merkle_roots_work_bytes(m, nb, width)));
        SHARD_HIP(c.b[6].ensure(nb * 32));
        PipeTail tail = [&](TxPipe& q, const uint8_t* d_hash, std::string& m2) -> int {
            const int rrc = launch_merkle_roots_batch(hasher, width, d_hash, boff.data(), nb, q.b[5].as<uint8_t>(),
                                                      q.b[6].as<uint8_t>(), q.compute);
            if (rrc) m2 = hip_msg(hipGetLastError(), "merkle roots launch");
            return rrc;
        };
        HostTxRange r = host_range(suite, pre, pre_off, sig, sig_off, lo, hi, txhash32, sender20, status);
        r.share = shards_on_device(devices, ndev, k, [&](int j) { return block_off[bl[j + 1]] > block_off[bl[j]]; });
        const int rc = tx_pipeline(c, r, tail, msg);
        if (rc) return rc;
        SHARD_HIP(hipMemcpyAsync(roots32 + 32 * b0, c.b[6].p, nb * 32, hipMemcpyDeviceToHost, c.copy));
        SHARD_HIP(hipStreamSynchronize(c.copy));
        return 0;
    });
}

}  // namespace

extern "C" {

int bcosgpu_init_devices(const int* devices, int ndev) { return check_set(devices, ndev); }

int bcosgpu_secp256k1_recover_batch_multi(const int* devices, int ndev, const uint8_t* hash32, const uint8_t* sig65,
                                          size_t n, uint8_t* pub64, uint8_t* addr20, uint8_t* ok) {
    if (n == 0) return check_set(devices, ndev);
    if (!hash32 || !sig65 || !ok) return api_set_err(BCOSGPU_E_ARG, "null pointer");
    return sig_multi(devices, ndev, kSigJobRecoverK1, n, hash32, sig65, 65, nullptr, pub64, addr20, ok);
}

int bcosgpu_sm2_verify_batch_multi(const int* devices, int ndev, const uint8_t* hash32, const uint8_t* sig128,
                                   size_t n, uint8_t* addr20, uint8_t* ok) {
    if (n == 0) return check_set(devices, ndev);
    if (!hash32 || !sig128 || !ok) return api_set_err(BCOSGPU_E_ARG, "null pointer");
    return sig_multi(devices, ndev, kSigJobVerifySM2, n, hash32, sig128, 128, nullptr, nullptr, addr20, ok);
}

int bcosgpu_verify_batch_multi(const int* devices, int ndev, int suite, const uint8_t* pub64, const uint8_t* hash32,
                               const uint8_t* sig, size_t sig_stride, size_t n, uint8_t* ok) {
    if (suite != BCOSGPU_SUITE_SECP256K1 && suite != BCOSGPU_SUITE_SM2) return api_set_err(BCOSGPU_E_ARG, "bad suite");
    if (sig_stride < 64 || sig_stride > 0xFFFFFFFFull) return api_set_err(BCOSGPU_E_ARG, "signature stride must be >= 64");
    if (n == 0) return check_set(devices, ndev);
    if (!pub64 || !hash32 || !sig || !ok) return api_set_err(BCOSGPU_E_ARG, "null pointer");
    return sig_multi(devices, ndev, suite == BCOSGPU_SUITE_SM2 ? kSigJobVerifySM2 : kSigJobVerifyK1, n, hash32, sig,
                     sig_stride, pub64, nullptr, nullptr, ok);
}

int bcosgpu_tx_verify_batch_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                                  const uint8_t* sig, const uint64_t* sig_off, size_t n, uint8_t* txhash32,
                                  uint8_t* sender20, uint8_t* status) {
    return tx_multi(devices, ndev, suite, pre, pre_off, sig, sig_off, n, 2, txhash32, sender20, status, nullptr);
}

int bcosgpu_block_verify_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                               const uint8_t* sig, const uint64_t* sig_off, size_t n, int width, uint8_t* txhash32,
                               uint8_t* sender20, uint8_t* status, uint8_t* root32) {
    if (!root32) return api_set_err(BCOSGPU_E_ARG, "null root pointer");
    return tx_multi(devices, ndev, suite, pre, pre_off, sig, sig_off, n, width, txhash32, sender20, status, root32);
}

int bcosgpu_blocks_verify_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                                const uint8_t* sig, const uint64_t* sig_off, const uint64_t* block_off, size_t nblocks,
                                int width, uint8_t* txhash32, uint8_t* sender20, uint8_t* status, uint8_t* roots32) {
    return blocks_multi(devices, ndev, suite, pre, pre_off, sig, sig_off, block_off, nblocks, width, txhash32, sender20,
                        status, roots32);
}

int bcosgpu_merkle_root_multi(const int* devices, int ndev, int hasher, int width, const uint8_t* leaves32, size_t n,
                              uint8_t* root32) {
    if (hasher != BCOSGPU_KECCAK256 && hasher != BCOSGPU_SM3) return api_set_err(BCOSGPU_E_ARG, "bad hasher");
    if (width < 2 || width > 64) return api_set_err(BCOSGPU_E_ARG, "width must be in [2, 64]");
    if (n == 0) return api_set_err(BCOSGPU_E_EMPTY, "Empty input");  // Merkle.h:172-175
    if (!leaves32 || !root32) return api_set_err(BCOSGPU_E_ARG, "null pointer");
    if (int rc = check_set(devices, ndev)) return rc;
    if (n == 1) {  // Merkle.h:177-182: the single leaf
        std::memcpy(root32, leaves32, 32);
        return 0;
    }
    enable_peers(devices, ndev);
    const Plan p = make_plan(n, ndev, width);
    std::vector<ShardCtx*> ctx = contexts(devices, ndev);
    ShardCtx* top = shard_ctx(devices[0], -1);
    std::vector<ShardCtx*> all = ctx;
    all.push_back(top);
    auto locks = lock_all(all);
    std::vector<const uint8_t*> frontier(ndev, nullptr);
    int rc = run_shards(ndev, [&](int k, std::string& msg) -> int {
        const uint64_t lo = p.lo[k], m = p.hi[k] - p.lo[k];
        if (!m) return 0;
        ShardCtx* c = ctx[k];
        DeviceGuard dg(c->device);
        SHARD_HIP(dg.err);
        SHARD_HIP(ensure_stream(c));
        SHARD_HIP(c->b[0].ensure(m * 32));
        SHARD_HIP(hipMemcpyAsync(c->b[0].p, leaves32 + 32 * lo, m * 32, hipMemcpyHostToDevice, c->stream));
        if (p.levels > 0) {
            SHARD_HIP(c->b[7].ensure(64 * ((m + width - 1) / width)));
            SHARD_HIP(c->b[8].ensure(32 * p.count(k)));
            const int lrc = launch_merkle_levels(hasher, width, c->b[0].as<uint8_t>(), m, p.levels,
                                                 c->b[7].as<uint8_t>(), c->b[8].as<uint8_t>(), c->stream);
            if (lrc) {
                msg = hip_msg(hipGetLastError(), "merkle frontier launch");
                return lrc;
            }
            frontier[k] = c->b[8].as<uint8_t>();
        } else {
            frontier[k] = c->b[0].as<uint8_t>();
        }
        SHARD_HIP(hipStreamSynchronize(c->stream));
        return 0;
    });
    if (rc) return rc;
    return gather_root(devices, ndev, p, frontier, hasher, width, top, root32);
}

}  // extern "C"
