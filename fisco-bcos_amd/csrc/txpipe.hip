// txpipe.hip -- the host-pointer tx-verify batches (bcosgpu_tx_verify_batch, the device-set shards of
// multi.hip) as a copy / compute pipeline.  The reference hands its batch sites host memory
// (TransactionSync.cpp:516-548 verifies a downloaded vector of transactions, BlockImpl.h:111-154 roots
// the block's hashes), so every such call pays PCIe both ways.  Measured on MI355X
// (tools/copybench.hip, profiles/r06_copybench.json): a pageable hipMemcpyAsync reaches the pinned rate
// (~56 GB/s) from ~27 MB up, returns only when its data has moved, and overlaps a kernel running on
// another stream.  So a batch is cut into chunks of one full round of the one-lane kernel at occupancy 2
// (512 txs per CU); while chunk k's kernel runs, the host thread copies chunk k+1 in and chunk k-1's
// results out, and only the first chunk's upload and the last chunk's download stay exposed.  Chunks
// alternate between two compute streams, so a chunk's kernel can start in the previous one's tail.
//
//  - Device buffers hold the whole range, so no chunk ever overwrites a buffer in use: chunk k's inputs go
//    to their final place, its kernel reads them through the range's own offsets (the device preimage
//    pointer is pre_off[lo] bytes before the buffer, so offsets need no host rebasing), its outputs land
//    at k's rows.
//  - Large batches: pageable H2D straight from the caller on the copy stream (the host blocks while they
//    move, i.e. while the previous chunk computes), an event, the chunk's compute stream waits on it;
//    once chunk k-1's kernel event has completed, pageable D2H straight into the caller's arrays (so no
//    copy waits on the GPU while holding the host thread).
//  - Small batches (<= 65536 txs, one launch: C2's 10k): staged through pinned memory on one stream, one
//    DMA in, one DMA of the outputs back (three pageable D2H of a 10k batch cost ~65 us).
//  - Pipelines come from a per-device pool: concurrent callers (the reference's verifier pools,
//    TxPool.h:48-49) each get their own streams and buffers, so their round trips overlap instead of
//    serialising behind one workspace mutex.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>
#include <sched.h>
#include "engine.h"

namespace bcosgpu {

hipError_t PipeBuf::ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    const hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
}

hipError_t PipeHostBuf::ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = hd = nullptr;
    cap = 0;
    const size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&hd, p, 0);
    if (e == hipSuccess) cap = want;
    return e;
}

namespace {

std::mutex g_pool_mu;
std::vector<std::vector<TxPipe*>> g_free;  // per device; pipes are never freed (no teardown races)

struct DevGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

hipError_t ensure_events(TxPipe& p, size_t need) {
    while (p.ev.size() < need) {
        hipEvent_t e;
        const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return r;
        p.ev.push_back(e);
    }
    return hipSuccess;
}

#define PIPE_HIP(call)                                               \
    do {                                                             \
        const hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) {                                      \
            msg = std::string(#call) + ": " + hipGetErrorString(e_); \
            return BCOSGPU_E_HIP;                                    \
        }                                                            \
    } while (0)

}  // namespace

TxPipe* tx_pipe_acquire(int device) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        if (device >= 0 && static_cast<size_t>(device) < g_free.size() && !g_free[device].empty()) {
            TxPipe* p = g_free[device].back();
            g_free[device].pop_back();
            return p;
        }
    }
    DevGuard dg(device);
    if (dg.err != hipSuccess) return nullptr;
    TxPipe* p = new TxPipe();
    p->device = device;
    if (hipStreamCreateWithFlags(&p->compute, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&p->compute2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;  // (a pipe without streams is dropped; the caller reports the failure)
    }
    return p;
}

void tx_pipe_release(TxPipe* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (g_free.size() <= static_cast<size_t>(p->device)) g_free.resize(p->device + 1);
    g_free[p->device].push_back(p);
}

uint64_t tx_pipe_chunk(uint64_t m, int share) {
    // BCOSGPU_PIPE_CHUNK (read per call; a test hook): force a chunk size, so chunk boundaries can be
    // tested at oracle-sized batches
    if (const char* e = std::getenv("BCOSGPU_PIPE_CHUNK")) {
        const long long v = std::atoll(e);
        if (v > 0) return std::min<uint64_t>(m, std::max<uint64_t>(static_cast<uint64_t>(v), (m + 4095) / 4096));
    }
    const uint64_t cus = static_cast<uint64_t>(cu_count());
    // one round of the occupancy-2 one-lane kernel, split between the shards sharing the device (two
    // shards on {0, 0} with half rounds: C4 68.5M against 67.9M tx/s with whole ones,
    // profiles/r06_devset_chunk_ab.json)
    const uint64_t c = 512 * cus / static_cast<uint64_t>(share < 1 ? 1 : share);
    // below two rounds one launch: its kernel choice beats chunks (two co-running halves of C2's 10k
    // trio round measured 0.604 ms against 0.557 for one launch, profiles/r06_hostpath_probe.json: the
    // second half's launch waits for its inputs and its trio round is as long as the whole batch's)
    return m >= 2 * c ? c : m;
}

namespace {
// The small path's host work -- the offsets check and the gather into pinned staging, the copy of the
// outputs back -- split over the calling thread and a few persistent helper threads: on one core the
// 2.3 MB of C2's 10k-tx inputs take ~47 us to copy into pinned memory (a quarter of the call's host time;
// threads spawned per call cost more than they save).  One call at a time uses the helpers; a concurrent
// caller works on its own thread.  BCOSGPU_PIPE_COPY_THREADS = helper count (default 3; 0: the caller
// alone), read once.
struct CopySeg {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};

void copy_range(const CopySeg* s, int nseg, size_t a, size_t b) {  // bytes [a, b) of the segments' concatenation
    size_t base = 0;
    for (int k = 0; k < nseg && base < b; base += s[k].n, ++k) {
        const size_t lo = std::max(a, base), hi = std::min(b, base + s[k].n);
        if (lo < hi) std::memcpy(s[k].dst + (lo - base), s[k].src + (lo - base), hi - lo);
    }
}

class HostPool {
public:
    static HostPool& get() {
        static HostPool* p = new HostPool();  // never destroyed: its threads live as long as the process
        return *p;
    }
    // fn(part, parts) for part = 0 .. parts - 1, part 0 on the calling thread; parts = 1 (the caller alone)
    // when `wide` is false, there are no helpers or another caller has them
    void run(const std::function<void(int, int)>& fn, bool wide) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!wide || helpers_ == 0 || !busy.owns_lock()) {
            fn(0, 1);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            left_.store(helpers_, std::memory_order_relaxed);
            ++gen_;
        }
        cv_.notify_all();
        fn(0, helpers_ + 1);
        while (left_.load(std::memory_order_acquire) != 0) sched_yield();
    }

private:
    HostPool() {
        const char* e = std::getenv("BCOSGPU_PIPE_COPY_THREADS");
        helpers_ = e ? std::max(0, std::min(15, std::atoi(e))) : 3;
        for (int i = 0; i < helpers_; ++i) std::thread([this, i] { worker(i + 1); }).detach();
    }
    void worker(int part) {
        uint64_t seen = 0;
        while (true) {
            const std::function<void(int, int)>* fn;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                fn = fn_;
            }
            (*fn)(part, helpers_ + 1);
            left_.fetch_sub(1, std::memory_order_release);
        }
    }
    int helpers_ = 0;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_;
    uint64_t gen_ = 0;
    const std::function<void(int, int)>* fn_ = nullptr;
    std::atomic<int> left_{0};
};

// One launch of a small batch (<= 65536 txs, one chunk), staged through pinned memory on ONE stream (no
// cross-stream events: an event wait added ~16 us before the kernel started).  Device layout =
// pinned layout: [preimages | signatures | pad | pre_off[m+1] | sig_off[m+1]] and the outputs
// [txhash | sender | status].  The host gathers everything into the staging buffer and sends it as ONE
// DMA (two DMAs -- the preimages' started while the rest was gathered -- measured an ~9 us gap between
// them in the copy queue, profiles/r06_pipe_trace.txt); kernel, the follow-on tail, one D2H of the
// outputs, one synchronisation, three host copies out.
int tx_small(TxPipe& p, const HostTxRange& t, const PipeTail& tail, std::string& msg) {
    const uint64_t lo = t.lo, hi = t.hi, m = hi - lo;
    const uint64_t pb = t.pre_off[lo], pbytes = t.pre_off[hi] - pb;
    const uint64_t sb = t.sig_off[lo], sbytes = t.sig_off[hi] - sb;
    const uint64_t spo = (pbytes + sbytes + 15) & ~7ull, sso = spo + 8 * (m + 1), total = sso + 8 * (m + 1);
    PIPE_HIP(p.b[0].ensure(total));
    PIPE_HIP(p.b[4].ensure(53 * m + 8));
    PIPE_HIP(p.hin.ensure(total));
    PIPE_HIP(p.host.ensure(53 * m));
    uint8_t* h = p.hin.as<uint8_t>();
    uint8_t* d = p.b[0].as<uint8_t>();
    hipStream_t st = p.compute;
    // each part checks its share of the offsets (nothing is launched unless all pass; the copy spans the
    // range's endpoints, checked by tx_pipeline, so it is safe either way) and gathers its share of bytes
    const CopySeg segs[4] = {{h, t.pre + pb, pbytes},
                             {h + pbytes, t.sig + sb, sbytes},
                             {h + spo, reinterpret_cast<const uint8_t*>(t.pre_off + lo), 8 * (m + 1)},
                             {h + sso, reinterpret_cast<const uint8_t*>(t.sig_off + lo), 8 * (m + 1)}};
    const size_t gather = pbytes + sbytes + 16 * (m + 1);
    std::atomic<bool> bad{false};
    HostPool::get().run(
        [&](int part, int parts) {
            for (uint64_t i = lo + m * part / parts, e = lo + m * (part + 1) / parts; i < e; ++i)
                if (t.pre_off[i + 1] < t.pre_off[i] || t.sig_off[i + 1] < t.sig_off[i] ||
                    t.pre_off[i + 1] - t.pre_off[i] > 0xFFFFFFFFull) {
                    bad.store(true, std::memory_order_relaxed);
                    break;
                }
            copy_range(segs, 4, gather * part / parts, gather * (part + 1) / parts);
        },
        gather >= (256u << 10));
    if (bad.load()) {
        msg = "offsets must be non-decreasing";
        return BCOSGPU_E_ARG;
    }
    PIPE_HIP(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, st));
    // without a tail the kernel writes its outputs straight into the mapped pinned buffer (no D2H copy and
    // no second wait on the copy engine); a tail reads the hashes on the device.  BCOSGPU_PIPE_ZCOUT=0
    // keeps the device outputs and one D2H (A/B hook, read once)
    static const bool zc_env = [] {
        const char* e = std::getenv("BCOSGPU_PIPE_ZCOUT");
        return !(e && e[0] == '0');
    }();
    const bool zc = !tail && zc_env;
    uint8_t* d_out = zc ? static_cast<uint8_t*>(p.host.hd) : p.b[4].as<uint8_t>();
    const int lrc = launch_tx_verify(t.suite, d - pb, reinterpret_cast<const uint64_t*>(d + spo), d + pbytes - sb,
                                     reinterpret_cast<const uint64_t*>(d + sso), m, d_out, d_out + 32 * m,
                                     d_out + 52 * m, st);
    if (lrc) {
        msg = std::string("tx verify launch: ") + hipGetErrorString(hipGetLastError());
        return lrc;
    }
    if (tail)
        if (int rc = tail(p, d_out, msg)) return rc;
    uint8_t* o = p.host.as<uint8_t>();
    if (!zc) PIPE_HIP(hipMemcpyAsync(o, d_out, 53 * m, hipMemcpyDeviceToHost, st));
    PIPE_HIP(hipStreamSynchronize(st));
    const CopySeg outs[3] = {{t.txhash32 + 32 * lo, o, 32 * m}, {t.sender20 + 20 * lo, o + 32 * m, 20 * m},
                             {t.status + lo, o + 52 * m, m}};
    HostPool::get().run([&](int part, int parts) { copy_range(outs, 3, 53 * m * part / parts, 53 * m * (part + 1) / parts); },
                        53 * m >= (256u << 10));
    return 0;
}
}  // namespace

int tx_pipeline(TxPipe& p, const HostTxRange& t, const PipeTail& tail, std::string& msg) {
    const uint64_t lo = t.lo, hi = t.hi, m = hi - lo;
    if (m == 0) return 0;
    // offsets are validated chunk by chunk, right before the chunk is sent (for 1M txs the 16 MB of offsets
    // take ~0.5 ms to check: that check now overlaps the previous chunk's kernel); the endpoints size the
    // device buffers, so they are checked first
    if (t.pre_off[hi] < t.pre_off[lo] || t.sig_off[hi] < t.sig_off[lo]) {
        msg = "offsets must be non-decreasing";
        return BCOSGPU_E_ARG;
    }
    const uint64_t chunk = tx_pipe_chunk(m, t.share);
    bool small = m <= 65536 && chunk == m;
    if (const char* e = std::getenv("BCOSGPU_PIPE_STAGED")) small = small && e[0] != '0';  // A/B hook
    if (small) return tx_small(p, t, tail, msg);
    const uint64_t pb = t.pre_off[lo], pbytes = t.pre_off[hi] - pb;
    const uint64_t sb = t.sig_off[lo], sbytes = t.sig_off[hi] - sb;
    // outputs contiguous: txhash [m][32] | sender [m][20] | status [m]  (sender stays 4-byte aligned)
    PIPE_HIP(p.b[0].ensure(pbytes + 8));
    PIPE_HIP(p.b[1].ensure((m + 1) * 8));
    PIPE_HIP(p.b[2].ensure(sbytes + 8));
    PIPE_HIP(p.b[3].ensure((m + 1) * 8));
    PIPE_HIP(p.b[4].ensure(53 * m + 8));
    // chunk boundaries: a quarter-round head chunk first (its upload is the pipeline's exposed start; its
    // kernel is less efficient, but the next chunk's kernel fills the rest of the GPU beside it on the
    // other compute stream), then whole rounds.  Not for a shard sharing its device with another shard of
    // the call (t.share > 1): there the other shard's first chunk already fills the GPU, and the head's
    // partial round only adds a launch (C5 on {0,0}: 71.6M tx/s without it, 68.5M with it;
    // profiles/r06_devset_head_ab.json).  BCOSGPU_PIPE_HEAD=0/1 forces it off/on (A/B hook).
    std::vector<uint64_t> cb{0};
    {
        const char* he = std::getenv("BCOSGPU_PIPE_HEAD");
        const bool want = he && (he[0] == '0' || he[0] == '1') ? he[0] == '1' : t.share <= 1;
        const bool head = chunk < m && !std::getenv("BCOSGPU_PIPE_CHUNK") && want;
        if (head) cb.push_back(chunk / 4);
        // a shard sharing its device takes its partial chunk FIRST (BCOSGPU_PIPE_REMFIRST=0/1 forces it
        // off/on): its small kernel then overlaps the next chunks, where as the last chunk it ran
        // alone at partial occupancy once the other shard had finished (a 1M C4 block on {0, 0}: ~1 ms of a
        // lone 41k-tx kernel, tools/trace_timeline.py over tools/pipe_trace.py devset; read per call, as
        // BCOSGPU_PIPE_HEAD)
        const char* re = std::getenv("BCOSGPU_PIPE_REMFIRST");
        const int remfirst_env = re && (re[0] == '0' || re[0] == '1') ? re[0] - '0' : -1;
        const bool remfirst = !head && chunk < m && m % chunk && (remfirst_env >= 0 ? remfirst_env == 1 : t.share > 1);
        if (remfirst) cb.push_back(m % chunk);
        while (cb.back() < m) cb.push_back(std::min(m, cb.back() + chunk));
    }
    const uint64_t nchunks = cb.size() - 1;
    PIPE_HIP(ensure_events(p, 2 * nchunks));
    // device views of the whole range: the byte buffers shifted back by the range's first offset, so the
    // caller's offsets index them directly
    const uint8_t* d_pre = p.b[0].as<uint8_t>() - pb;
    const uint8_t* d_sig = p.b[2].as<uint8_t>() - sb;
    uint64_t* d_po = p.b[1].as<uint64_t>();
    uint64_t* d_so = p.b[3].as<uint64_t>();
    uint8_t* d_out = p.b[4].as<uint8_t>();
    uint8_t *d_hash = d_out, *d_snd = d_out + 32 * m, *d_st = d_out + 52 * m;
    hipStream_t cs[2] = {p.compute, p.compute2};
    if (const char* e = std::getenv("BCOSGPU_PIPE_STREAMS"))  // A/B hook: 1 = every chunk on one stream
        if (e[0] == '1') cs[1] = p.compute;
    auto drain = [&](uint64_t k) -> int {  // the large path: chunk k's outputs once its kernel is done
        const uint64_t a = cb[k], e = cb[k + 1], c = e - a;
        PIPE_HIP(hipEventSynchronize(p.ev[2 * k + 1]));
        PIPE_HIP(hipMemcpyAsync(t.txhash32 + 32 * (lo + a), d_hash + 32 * a, 32 * c, hipMemcpyDeviceToHost, p.copy));
        PIPE_HIP(hipMemcpyAsync(t.sender20 + 20 * (lo + a), d_snd + 20 * a, 20 * c, hipMemcpyDeviceToHost, p.copy));
        PIPE_HIP(hipMemcpyAsync(t.status + lo + a, d_st + a, c, hipMemcpyDeviceToHost, p.copy));
        return 0;
    };
    for (uint64_t k = 0; k < nchunks; ++k) {
        const uint64_t a = cb[k], e = cb[k + 1], c = e - a;
        const uint64_t ga = lo + a, ge = lo + e;  // the chunk in the caller's indexing
        for (uint64_t i = ga; i < ge; ++i)
            if (t.pre_off[i + 1] < t.pre_off[i] || t.sig_off[i + 1] < t.sig_off[i] ||
                t.pre_off[i + 1] - t.pre_off[i] > 0xFFFFFFFFull || t.pre_off[i + 1] > t.pre_off[hi] ||
                t.sig_off[i + 1] > t.sig_off[hi]) {
                (void)hipStreamSynchronize(cs[0]);  // the chunks already launched finish before the error returns
                (void)hipStreamSynchronize(cs[1]);
                (void)hipStreamSynchronize(p.copy);
                msg = "offsets must be non-decreasing";
                return BCOSGPU_E_ARG;
            }
        const uint64_t p0 = t.pre_off[ga], p1 = t.pre_off[ge], s0 = t.sig_off[ga], s1 = t.sig_off[ge];
        hipStream_t st = cs[k & 1];
        // pageable copies straight from the caller (they return once their data has moved)
        if (p1 > p0)
            PIPE_HIP(hipMemcpyAsync(p.b[0].as<uint8_t>() + (p0 - pb), t.pre + p0, p1 - p0, hipMemcpyHostToDevice,
                                    p.copy));
        if (s1 > s0)
            PIPE_HIP(hipMemcpyAsync(p.b[2].as<uint8_t>() + (s0 - sb), t.sig + s0, s1 - s0, hipMemcpyHostToDevice,
                                    p.copy));
        PIPE_HIP(hipMemcpyAsync(d_po + a, t.pre_off + ga, (c + 1) * 8, hipMemcpyHostToDevice, p.copy));
        PIPE_HIP(hipMemcpyAsync(d_so + a, t.sig_off + ga, (c + 1) * 8, hipMemcpyHostToDevice, p.copy));
        PIPE_HIP(hipEventRecord(p.ev[2 * k], p.copy));
        PIPE_HIP(hipStreamWaitEvent(st, p.ev[2 * k], 0));
        const int lrc = launch_tx_verify(t.suite, d_pre, d_po + a, d_sig, d_so + a, c, d_hash + 32 * a, d_snd + 20 * a,
                                         d_st + a, st);
        if (lrc) {
            msg = std::string("tx verify launch: ") + hipGetErrorString(hipGetLastError());
            return lrc;
        }
        PIPE_HIP(hipEventRecord(p.ev[2 * k + 1], st));
        if (k + 1 == nchunks) {
            // compute stream 0 joins the other stream's last chunk, then the follow-on kernels over the
            // whole range's hashes (roots, frontier)
            if (nchunks >= 2) {
                const uint64_t j = (k & 1) ? k : k - 1;  // the last chunk that ran on stream 1
                PIPE_HIP(hipStreamWaitEvent(cs[0], p.ev[2 * j + 1], 0));
            }
            if (tail)
                if (int rc = tail(p, d_hash, msg)) return rc;
        }
        if (k >= 1)
            if (int rc = drain(k - 1)) return rc;
    }
    if (int rc = drain(nchunks - 1)) return rc;
    PIPE_HIP(hipStreamSynchronize(p.copy));
    PIPE_HIP(hipStreamSynchronize(cs[0]));
    PIPE_HIP(hipStreamSynchronize(cs[1]));
    return 0;
}

}  // namespace bcosgpu
