// coalesce.hip -- per-device coalescing of the host-pointer signature calls.
//
// The reference verifies one signature per call on its hot admission path: TxPool's submitter pool
// (hardware_concurrency threads, TxPool.h:48-49) runs TxValidator::verify -> Transaction::verify ->
// SignatureCrypto::recover once per transaction (TxValidator.cpp:56, Transaction.h:68-82).  A kernel
// launch per call would serialise those threads behind one latency-bound launch each.  Instead every
// host-pointer recover / verify call (single or batched) becomes a job in its device's queue; a caller
// that finds a free launch slot takes EVERY queued job of its kind (up to kMaxBatch items) and runs them
// as one batch -- assemble into pinned staging, one H2D copy, one launch (the same rounds x latency
// kernel choice as the tx path, ecc_txv.hip launch_verify), one D2H copy, synchronise, scatter -- while
// the other callers sleep, each on its own job (see notify_job and lockfree_arrivals).  No dispatcher
// thread: the callers themselves lead batches
// (leader / follower), so nothing runs when nobody calls and nothing needs shutting down.  Up to
// slots_in_use() batches can be in flight per device at once, each on its own stream: small
// latency-bound batches occupy a few CUs each, so they overlap on the device instead of queueing.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <vector>
#include <cstdlib>
#include <cstring>
#include <linux/futex.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>
#include "engine.h"

namespace bcosgpu {
namespace {

constexpr int kMaxSlots = 16;
constexpr size_t kMaxBatch = 65536;

// batches in flight per device: 4 (GPU_MAX_HW_QUEUES' default), BCOSGPU_COALESCE_SLOTS = 1..16 to tune
int slots_in_use() {
    static const int n = [] {
        const char* e = getenv("BCOSGPU_COALESCE_SLOTS");
        const int v = e ? atoi(e) : 4;
        return v < 1 ? 1 : v > kMaxSlots ? kMaxSlots : v;
    }();
    return n;
}

// How a leader waits for its batch (BCOSGPU_COALESCE_WAIT, read once): 0 hipStreamSynchronize (the
// runtime spins on the completion signal), 1 a blocking-sync event (the thread sleeps until the GPU's
// interrupt), 2 poll the event and yield the CPU between polls, 3 poll the event and sleep ~15 us between
// polls (1 us timer slack on the leader thread), 4 (default) as 3 until 25 us before the batch's expected
// end (a running average of the GPU time of the last batches of its kind, kernel family -- registered-key
// or not -- and size class), then poll without sleeping.
// hipStreamSynchronize and even a blocking-sync event spin on the CPU for a batch's whole ~0.13-0.35 ms
// (one core per batch in flight: a lone caller's process used 1.0 core); mode 4 keeps the spin's latency
// (p50 132.1 vs 132.0 us for one caller) on 0.26 of a core, and 1.6 / 3.9 cores instead of 4.1 / 6.2 at
// 16 / 64 callers -- cores a node's executor and consensus threads get back -- for throughput within
// 2-5 % (tools/callbench_sweep.py, profiles/r06_coalesce_wait_ab.jsonl)
int wait_mode() {
    static const int m = [] {
        const char* e = getenv("BCOSGPU_COALESCE_WAIT");
        const int v = e ? atoi(e) : 4;
        return v < 0 || v > 4 ? 4 : v;
    }();
    return m;
}

// Batches in flight: slots_in_use() while fewer than kDeepCallers callers are inside the device's queue,
// 2 beyond (with ~256 submitter threads on the box's 16 cores more concurrent leaders only add host CPU
// -- polling leaders, smaller batches, more wake-ups -- to a process already at its CPU quota:
// tools/callbench_sweep.py, profiles/r06_callbench_slots.jsonl: secp256k1 at 256 threads 245k calls/s
// with 4 slots, 347k with 2; at 16 / 64 threads 4 slots stay ahead, 80k / 266k against 72k / 254k;
// the cap against none on one box, profiles/r06_coalesce_deep_ab.json: 257-273k against 187-219k, p99
// 2 ms against 60 ms).  Measured before the lock-free arrivals below; with them the CPU is no longer the
// bound, the cap is neutral for secp256k1 and still worth ~6 % for SM2's longer batches at 256 threads
// (profiles/r06_coalesce_deep_ab2.json), so it stays.
// BCOSGPU_COALESCE_DEEP = the caller count (default 128; 0 keeps slots_in_use() always), read once.
int deep_callers() {
    static const int n = [] {
        const char* e = getenv("BCOSGPU_COALESCE_DEEP");
        return e ? atoi(e) : 128;
    }();
    return n;
}

struct Slot {
    int index = 0;
    bool busy = false;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // wait modes 1 and 2
    uint8_t* h_in = nullptr;  // pinned, device-mapped staging
    uint8_t* h_out = nullptr;
    uint8_t* hd_in = nullptr;  // their device addresses (zero-copy small batches)
    uint8_t* hd_out = nullptr;
    size_t h_in_cap = 0, h_out_cap = 0;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    size_t d_in_cap = 0, d_out_cap = 0;
};

// Where a coalesced call's time goes (bcosgpu_coalesce_stats): per device, summed over calls / batches,
// in nanoseconds.  All updated under the queue mutex except the batch phases (one leader each, atomics).
enum CoalesceStat {
    kStBatches = 0,   // batches launched
    kStJobs,          // calls completed
    kStItems,         // signatures
    kStQueueNs,       // per call: enqueue -> its batch taken by a leader
    kStLeadNs,        // per batch: the leader's host work before the launch (staging, key lookup)
    kStGpuNs,         // per batch: first launch -> results synchronised (kernel + copies + queue)
    kStScatterNs,     // per batch: results copied out to the callers
    kStWakeNs,        // per woken follower / leader: notify -> running again (scheduler latency)
    kStWakes,         // wake-ups counted in kStWakeNs
    kStLockNs,        // per call: waiting for the queue mutex on entry
    kStCount
};

struct DeviceQueue {
    std::mutex mu;
    std::atomic<int> callers{0};  // callers inside coalesced_run on this device
    // arrivals push their job here without the mutex; whoever holds the mutex moves them to pending
    std::atomic<SigJob*> incoming{nullptr};
    std::atomic<int> idle{0};     // slots free within the current cap (written under mu)
    uint64_t next_seq = 0;
    std::deque<SigJob*> pending[kSigJobKinds];
    Slot slots[kMaxSlots];
    std::atomic<uint64_t> stat[kStCount];
    DeviceQueue() {
        for (auto& x : stat) x.store(0, std::memory_order_relaxed);
        idle.store(slots_in_use(), std::memory_order_relaxed);
    }
};

inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

std::mutex g_qmu;
DeviceQueue* g_queues[64] = {};  // never freed: no teardown races with the HIP runtime at exit

DeviceQueue* queue_of(int device) {
    std::lock_guard<std::mutex> g(g_qmu);
    if (!g_queues[device]) {
        g_queues[device] = new DeviceQueue();
        for (int k = 0; k < kMaxSlots; ++k) g_queues[device]->slots[k].index = k;
    }
    return g_queues[device];
}

size_t grow(size_t want) { return want < 65536 ? 65536 : want + want / 4; }

hipError_t ensure_pinned(uint8_t*& p, uint8_t*& dp, size_t& cap, size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    cap = 0;
    const size_t want = grow(bytes);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&dp), p, 0);
    if (e == hipSuccess) cap = want;
    return e;
}

// Batches up to this many items are read and written by the kernel in place, in the mapped staging
// (zero-copy: no copy dispatches, which cost a latency-bound single call ~2 x 20-60 us of queue time);
// larger ones are copied by the DMA engines.
constexpr size_t kZeroCopyMax = 2048;

hipError_t ensure_dev(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = grow(bytes);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want);
    if (e == hipSuccess) cap = want;
    return e;
}

// Bytes per item of the staged input and output of each job kind.
//   recover secp256k1: in  hash[32] .. | sig[65] ..          out pub[64] .. | addr[20] .. | ok ..
//   verify SM2:        in  hash[32] .. | r||s||pub[128] ..   out addr[20] .. | ok ..
//   verify secp256k1:  in  pub[64] .. | hash[32] .. | r||s[64] ..   out ok ..
constexpr size_t kInPer[kSigJobKinds] = {32 + 65, 32 + 128, 64 + 32 + 64};
constexpr size_t kOutPer[kSigJobKinds] = {64 + 20 + 1, 20 + 1, 1};

int fail(std::vector<SigJob*>& batch, int rc, const std::string& msg) {
    for (SigJob* j : batch) {
        j->rc = rc;
        j->err = msg;
    }
    return rc;
}

#define BATCH_HIP(call)                                                                        \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) return fail(batch, BCOSGPU_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

// One coalesced launch for `batch` (all of one kind) on `slot` of `device`.
int run_batch(int device, int kind, Slot& slot, std::vector<SigJob*>& batch, std::atomic<uint64_t>* stat) {
    const int64_t t_lead = now_ns();
    int64_t t_launch = 0, t_synced = 0;
    size_t n = 0;
    bool want_addr = false, want_pub = false;
    for (SigJob* j : batch) {
        n += j->n;
        want_addr = want_addr || j->out_addr20;
        want_pub = want_pub || j->out_pub64;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != device) BATCH_HIP(hipSetDevice(device));
    struct Restore {
        int prev, dev;
        ~Restore() {
            if (prev != dev) (void)hipSetDevice(prev);
        }
    } restore{prev, device};
    if (!slot.stream) {
        // Streams of one priority share a few hardware queues (GPU_MAX_HW_QUEUES), and kernels on one
        // queue run in order, so slot k takes priority level k mod levels: each level brings its own
        // queues and the batches in flight really overlap (BCOSGPU_COALESCE_PRIO=0: all at the default).
        static const bool prio = !getenv("BCOSGPU_COALESCE_PRIO") || atoi(getenv("BCOSGPU_COALESCE_PRIO")) != 0;
        int least = 0, greatest = 0;
        if (prio) BATCH_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        const int levels = least >= greatest ? least - greatest + 1 : 1;
        BATCH_HIP(hipStreamCreateWithPriority(&slot.stream, hipStreamNonBlocking, least - slot.index % levels));
    }
    if (!slot.done && wait_mode() != 0)
        BATCH_HIP(hipEventCreateWithFlags(&slot.done, hipEventDisableTiming |
                                                          (wait_mode() == 1 ? hipEventBlockingSync : 0u)));
    // verify kinds stage the keys' cache slots (int32 per item) after the input (registered-key path)
    const bool verify = kind == kSigJobVerifyK1 || kind == kSigJobVerifySM2;
    const size_t slots_at = kInPer[kind] * n;
    const size_t in_bytes = slots_at + (verify ? 4 * n : 0), out_bytes = kOutPer[kind] * n;
    BATCH_HIP(ensure_pinned(slot.h_in, slot.hd_in, slot.h_in_cap, in_bytes));
    BATCH_HIP(ensure_pinned(slot.h_out, slot.hd_out, slot.h_out_cap, out_bytes));
    static const size_t zero_copy_max = [] {
        const char* e = getenv("BCOSGPU_COALESCE_ZEROCOPY");  // items; tuning
        return e ? static_cast<size_t>(atol(e)) : kZeroCopyMax;
    }();
    const bool zero_copy = n <= zero_copy_max;
    if (!zero_copy) {
        BATCH_HIP(ensure_dev(slot.d_in, slot.d_in_cap, in_bytes + 16));
        BATCH_HIP(ensure_dev(slot.d_out, slot.d_out_cap, out_bytes + 16));
    }
    // assemble the SoA input
    uint8_t* in = slot.h_in;
    size_t at = 0;
    for (SigJob* j : batch) {
        const size_t m = j->n;
        if (kind == kSigJobRecoverK1) {
            std::memcpy(in + 32 * at, j->hash32, 32 * m);
            uint8_t* s = in + 32 * n + 65 * at;
            if (j->sig_stride == 65) std::memcpy(s, j->sig, 65 * m);
            else for (size_t i = 0; i < m; ++i) std::memcpy(s + 65 * i, j->sig + j->sig_stride * i, 65);
        } else if (kind == kSigJobVerifySM2) {
            std::memcpy(in + 32 * at, j->hash32, 32 * m);
            uint8_t* s = in + 32 * n + 128 * at;
            if (!j->pub64 && j->sig_stride == 128) {
                std::memcpy(s, j->sig, 128 * m);
            } else {
                for (size_t i = 0; i < m; ++i) {
                    std::memcpy(s + 128 * i, j->sig + j->sig_stride * i, 64);
                    std::memcpy(s + 128 * i + 64, j->pub64 ? j->pub64 + 64 * i : j->sig + j->sig_stride * i + 64, 64);
                }
            }
        } else {
            std::memcpy(in + 64 * at, j->pub64, 64 * m);
            std::memcpy(in + 64 * n + 32 * at, j->hash32, 32 * m);
            uint8_t* s = in + 96 * n + 64 * at;
            for (size_t i = 0; i < m; ++i) std::memcpy(s + 64 * i, j->sig + j->sig_stride * i, 64);
        }
        at += m;
    }
    // every key of the batch registered (or promoted now): the registered-key kernel (ecc_keyed.hip)
    bool keyed = false;
    uint64_t gen = 0;
    const int vsuite = kind == kSigJobVerifySM2 ? BCOSGPU_SUITE_SM2 : BCOSGPU_SUITE_SECP256K1;
    if (verify) {
        const uint8_t* pubs = kind == kSigJobVerifySM2 ? in + 32 * n + 64 : in;
        // only calls that name their keys (SignatureCrypto::verify: the sealer path) promote keys; SM2 recover
        // (admission: the key is the sender's, embedded in the signature) only looks them up
        bool named = true;
        for (SigJob* j : batch) named = named && (kind == kSigJobVerifyK1 || j->pub64 != nullptr);
        const int krc = keyed_slots(vsuite, pubs, kind == kSigJobVerifySM2 ? 128 : 64, n,
                                    reinterpret_cast<int32_t*>(in + slots_at), false, &keyed, slot.stream, &gen, named);
        if (krc) keyed = false;  // a failed table build leaves the generic path
    }
    if (!zero_copy) BATCH_HIP(hipMemcpyAsync(slot.d_in, slot.h_in, in_bytes, hipMemcpyHostToDevice, slot.stream));
    const uint8_t* di = zero_copy ? slot.hd_in : slot.d_in;
    uint8_t* dout = zero_copy ? slot.hd_out : slot.d_out;
    t_launch = now_ns();
    for (int attempt = 0; attempt < 2; ++attempt) {
        int rc;
        if (keyed && kind == kSigJobVerifySM2)
            rc = launch_sig_verify_keyed(BCOSGPU_SUITE_SM2, reinterpret_cast<const int32_t*>(di + slots_at), di,
                                         di + 32 * n, 128, n, dout + 20 * n, want_addr ? dout : nullptr, slot.stream);
        else if (keyed)
            rc = launch_sig_verify_keyed(BCOSGPU_SUITE_SECP256K1, reinterpret_cast<const int32_t*>(di + slots_at),
                                         di + 64 * n, di + 96 * n, 64, n, dout, nullptr, slot.stream);
        else if (kind == kSigJobRecoverK1)
            rc = launch_secp256k1_recover(di, di + 32 * n, 65, n, want_pub ? dout : nullptr,
                                          want_addr ? dout + 64 * n : nullptr, dout + 84 * n, slot.stream);
        else if (kind == kSigJobVerifySM2)
            rc = launch_sm2_verify(di, di + 32 * n, 128, n, want_addr ? dout : nullptr, dout + 20 * n, slot.stream);
        else
            rc = launch_sig_verify(BCOSGPU_SUITE_SECP256K1, di, di + 64 * n, di + 96 * n, 64, n, dout, slot.stream);
        if (rc) {
            hipError_t e = hipGetLastError();
            return fail(batch, rc, std::string("signature batch launch failed: ") + hipGetErrorString(e));
        }
        if (!zero_copy)
            BATCH_HIP(hipMemcpyAsync(slot.h_out, slot.d_out, out_bytes, hipMemcpyDeviceToHost, slot.stream));
        if (wait_mode() == 0) {
            BATCH_HIP(hipStreamSynchronize(slot.stream));
        } else {
            BATCH_HIP(hipEventRecord(slot.done, slot.stream));
            if (wait_mode() == 1) {
                BATCH_HIP(hipEventSynchronize(slot.done));
            } else {
                static thread_local bool slack = false;
                if (wait_mode() >= 3 && !slack) {
                    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
                    slack = true;
                }
                // running average GPU time per (kind, registered-key kernel or not, batch size by powers of 2)
                static std::atomic<int64_t> expect[kSigJobKinds][2][18];
                int lg = 0;
                while (lg < 17 && (size_t{1} << (lg + 1)) <= n) ++lg;
                std::atomic<int64_t>& expect_ns = expect[kind][keyed ? 1 : 0][lg];
                const int64_t sleep_until = wait_mode() == 4 ? t_launch + expect_ns.load(std::memory_order_relaxed) - 25000
                                                             : INT64_MAX;
                const timespec nap{0, 15000};
                hipError_t qe;
                while ((qe = hipEventQuery(slot.done)) == hipErrorNotReady) {
                    if (wait_mode() == 2) sched_yield();
                    else if (now_ns() < sleep_until) nanosleep(&nap, nullptr);
                }
                BATCH_HIP(qe);
                if (wait_mode() == 4) {
                    const int64_t took = now_ns() - t_launch, e = expect_ns.load(std::memory_order_relaxed);
                    expect_ns.store(e == 0 ? took : e + (took - e) / 8, std::memory_order_relaxed);
                }
            }
        }
        // the key cache was cleared (bcosgpu_clear_keys) between the lookup and the launch: its slots may
        // have been rebuilt for other keys meanwhile, so this batch runs again on the generic kernels
        if (!keyed || keyed_generation(vsuite) == gen) break;
        keyed = false;
    }
    t_synced = now_ns();
    // scatter
    const uint8_t* out = slot.h_out;
    at = 0;
    for (SigJob* j : batch) {
        const size_t m = j->n;
        if (kind == kSigJobRecoverK1) {
            if (j->out_pub64) std::memcpy(j->out_pub64, out + 64 * at, 64 * m);
            if (j->out_addr20) std::memcpy(j->out_addr20, out + 64 * n + 20 * at, 20 * m);
            std::memcpy(j->out_ok, out + 84 * n + at, m);
        } else if (kind == kSigJobVerifySM2) {
            if (j->out_addr20) std::memcpy(j->out_addr20, out + 20 * at, 20 * m);
            std::memcpy(j->out_ok, out + 20 * n + at, m);
        } else {
            std::memcpy(j->out_ok, out + at, m);
        }
        j->rc = 0;
        at += m;
    }
    stat[kStBatches].fetch_add(1, std::memory_order_relaxed);
    stat[kStItems].fetch_add(n, std::memory_order_relaxed);
    stat[kStLeadNs].fetch_add(static_cast<uint64_t>(t_launch - t_lead), std::memory_order_relaxed);
    stat[kStGpuNs].fetch_add(static_cast<uint64_t>(t_synced - t_launch), std::memory_order_relaxed);
    stat[kStScatterNs].fetch_add(static_cast<uint64_t>(now_ns() - t_synced), std::memory_order_relaxed);
    return 0;
}

}  // namespace

// Wake-ups are targeted, never broadcast: a finished batch wakes its own jobs' owners, and for every
// free slot the owner of the oldest queued job (of any kind) to lead the next batch.  (A broadcast on
// every completion woke all callers -- 256 submitter threads on the box's 16 cores -- per batch: at
// 256 threads secp256k1 single calls fell to 30k/s with a p99 of 87 ms, profiles/r04_bench_first.json.)
// An owner sleeps on its job's own futex word, and a leader marks its batch's jobs done and wakes their
// owners AFTER releasing the device queue's mutex: at 256 callers on 16 cores, notifying ~20 owners under
// that mutex held it ~0.1 ms per batch and every new call queued behind it (tools/callbench_sweep.py,
// profiles/r06_callbench_sweep.json: lock wait 0.17 -> 0.75 ms per call when only the wait moved).  The
// word, not a mutex + condition variable: a notify under the job's mutex woke the owner only for it to
// block again on that mutex (two context switches per wake-up).  The notifier's last access to the job is
// the release fetch_or that publishes the bit (rc, outputs and t_notify are written before it); the
// FUTEX_WAKE after it names only the word's address, so an owner that has already seen the bit and
// returned (its SigJob gone) costs at most a spurious wake-up of whatever waits there later, which every
// futex waiter tolerates.
static constexpr uint32_t kSigWake = 1, kSigDone = 2;

static void futex_wait(std::atomic<uint32_t>& a, uint32_t v) {
    (void)syscall(SYS_futex, reinterpret_cast<uint32_t*>(&a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
static void futex_wake(uint32_t* a) {
    (void)syscall(SYS_futex, a, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

static void notify_job(SigJob* j, bool done, int64_t t) {
    uint32_t* word = reinterpret_cast<uint32_t*>(&j->wake);
    if (!done) j->woken = true;  // (under q.mu: wake_leaders)
    j->t_notify.store(t, std::memory_order_relaxed);
    j->wake.fetch_or(done ? kSigDone : kSigWake, std::memory_order_release);  // last access to *j
    futex_wake(word);
}

static int slots_now(const DeviceQueue& q) {
    const int deep = deep_callers();
    return deep > 0 && q.callers.load(std::memory_order_relaxed) >= deep ? std::min(2, slots_in_use()) : slots_in_use();
}

// Arrivals without the queue mutex (BCOSGPU_COALESCE_LOCKFREE, default 1, read once): a caller pushes its
// job on q.incoming and takes the mutex only when a slot is free (q.idle > 0); otherwise it sleeps at once,
// and every holder of the mutex moves the arrivals to pending first.  No arrival is stranded: a leader
// stores q.idle after freeing its slot and only then drains, while an arrival pushes and only then reads
// q.idle (all sequentially consistent), so either the leader's drain sees the job or the arrival sees the
// free slot and comes to lead.  At 256 submitter threads every arrival used to queue on the mutex (tens of
// us per call under the box's CPU quota, its holders preempted).
static bool lockfree_arrivals() {
    static const bool v = [] {
        const char* e = getenv("BCOSGPU_COALESCE_LOCKFREE");
        return !(e && e[0] == '0');
    }();
    return v;
}

static void refresh_idle(DeviceQueue& q) {  // under q.mu
    int free_slots = 0;
    for (int k = 0, cap = slots_now(q); k < cap; ++k) free_slots += !q.slots[k].busy;
    q.idle.store(free_slots, std::memory_order_seq_cst);
}

static void drain(DeviceQueue& q) {  // under q.mu: arrivals to pending, in arrival order
    SigJob* h = q.incoming.exchange(nullptr, std::memory_order_seq_cst);
    SigJob* fifo = nullptr;
    while (h) {
        SigJob* n = h->next;
        h->next = fifo;
        fifo = h;
        h = n;
    }
    for (SigJob* j = fifo; j; j = j->next) {
        j->queued = true;
        j->seq = q.next_seq++;
        q.pending[j->kind].push_back(j);
    }
}

static void wake_leaders(DeviceQueue& q) {  // under q.mu
    int free_slots = 0;
    for (int k = 0, cap = slots_now(q); k < cap; ++k) free_slots += !q.slots[k].busy;
    for (int pass = 0; pass < kSigJobKinds && free_slots > 0; ++pass) {
        // the kind whose front job has waited longest first (jobs carry their arrival order)
        SigJob* best = nullptr;
        for (int kd = 0; kd < kSigJobKinds; ++kd) {
            auto& pend = q.pending[kd];
            if (pend.empty() || pend.front()->woken) continue;
            if (!best || pend.front()->seq < best->seq) best = pend.front();
        }
        if (!best) return;
        notify_job(best, false, now_ns());
        --free_slots;
    }
}

int coalesced_run(int device, SigJob& job) {
    if (device < 0 || device >= 64 || job.kind < 0 || job.kind >= kSigJobKinds) {
        job.err = "bad device or job kind";
        return job.rc = BCOSGPU_E_ARG;
    }
    if (job.n == 0) return job.rc = 0;
    DeviceQueue& q = *queue_of(device);
    struct Inside {
        std::atomic<int>& c;
        explicit Inside(std::atomic<int>& x) : c(x) { c.fetch_add(1, std::memory_order_relaxed); }
        ~Inside() { c.fetch_sub(1, std::memory_order_relaxed); }
    } inside(q.callers);
    job.wake.store(0, std::memory_order_relaxed);
    job.queued = false;
    job.woken = false;
    job.t_notify.store(0, std::memory_order_relaxed);
    job.t_enq = now_ns();
    std::unique_lock<std::mutex> lk(q.mu, std::defer_lock);
    bool sleep_first = false;
    if (lockfree_arrivals()) {
        SigJob* h = q.incoming.load(std::memory_order_relaxed);
        do {
            job.next = h;
        } while (!q.incoming.compare_exchange_weak(h, &job, std::memory_order_seq_cst, std::memory_order_relaxed));
        sleep_first = q.idle.load(std::memory_order_seq_cst) == 0;  // every slot busy: a leader will drain
    }
    if (!sleep_first) {
        const int64_t t_call = now_ns();
        lk.lock();
        q.stat[kStLockNs].fetch_add(static_cast<uint64_t>(now_ns() - t_call), std::memory_order_relaxed);
        if (lockfree_arrivals()) {
            drain(q);
        } else {
            job.queued = true;
            job.seq = q.next_seq++;
            q.pending[job.kind].push_back(&job);
        }
    }
    // A caller leads only while its own job is still queued (a caller whose job is in flight just waits
    // for its batch to finish).
    while (true) {
        Slot* free_slot = nullptr;
        if (!sleep_first) {
            if (job.wake.load(std::memory_order_acquire) & kSigDone) return job.rc;  // (lk released on return)
            for (int k = 0, cap = slots_now(q); k < cap; ++k)
                if (!q.slots[k].busy) {
                    free_slot = &q.slots[k];
                    break;
                }
        }
        if (sleep_first || !free_slot || !job.queued) {
            if (!sleep_first) lk.unlock();
            sleep_first = false;
            uint32_t s;
            while (((s = job.wake.load(std::memory_order_acquire)) & (kSigWake | kSigDone)) == 0) futex_wait(job.wake, s);
            const int64_t tn = job.t_notify.exchange(0, std::memory_order_relaxed);
            if (tn) {  // a targeted wake-up: its scheduler latency
                q.stat[kStWakeNs].fetch_add(static_cast<uint64_t>(now_ns() - tn), std::memory_order_relaxed);
                q.stat[kStWakes].fetch_add(1, std::memory_order_relaxed);
            }
            if (s & kSigDone) return job.rc;
            job.wake.fetch_and(~kSigWake, std::memory_order_relaxed);
            lk.lock();
            drain(q);
            job.woken = false;  // (wake_leaders sets it under q.mu)
            continue;
        }
        // lead: take every queued job of this kind, oldest first, up to kMaxBatch items (at least one)
        drain(q);
        auto& pend = q.pending[job.kind];
        std::vector<SigJob*> batch;
        size_t items = 0;
        const int64_t t_take = now_ns();
        while (!pend.empty() && (batch.empty() || items + pend.front()->n <= kMaxBatch)) {
            items += pend.front()->n;
            pend.front()->queued = false;
            q.stat[kStQueueNs].fetch_add(static_cast<uint64_t>(t_take - pend.front()->t_enq), std::memory_order_relaxed);
            batch.push_back(pend.front());
            pend.pop_front();
        }
        free_slot->busy = true;
        refresh_idle(q);
        lk.unlock();
        // a host exception (std::bad_alloc from the staging vectors) fails this batch only: the slot is
        // released and every job of the batch is completed with the error, so no caller waits forever
        try {
            run_batch(device, job.kind, *free_slot, batch, q.stat);
        } catch (const std::exception& e) {
            fail(batch, BCOSGPU_E_HIP, std::string("signature batch failed on the host: ") + e.what());
        } catch (...) {
            fail(batch, BCOSGPU_E_HIP, "signature batch failed on the host");
        }
        lk.lock();
        free_slot->busy = false;
        refresh_idle(q);  // before the drain (see lockfree_arrivals)
        drain(q);
        wake_leaders(q);
        lk.unlock();
        const int64_t t_done = now_ns();
        bool mine = false;
        for (SigJob* j : batch) {
            if (j == &job) {
                mine = true;
                continue;
            }
            notify_job(j, true, t_done);  // j's owner may return (and j go away) once the bit is set
        }
        q.stat[kStJobs].fetch_add(batch.size(), std::memory_order_relaxed);
        if (mine) return job.rc;
        lk.lock();  // the batch was full before this caller's own job: lead or wait again
        drain(q);
    }
}

int coalesce_stats(int device, uint64_t* out, int n, int reset) {
    if (device < 0 || device >= 64 || !out) return BCOSGPU_E_ARG;
    DeviceQueue& q = *queue_of(device);
    for (int k = 0; k < kStCount; ++k) {
        const uint64_t v = reset ? q.stat[k].exchange(0, std::memory_order_relaxed) : q.stat[k].load(std::memory_order_relaxed);
        if (k < n) out[k] = v;
    }
    return 0;
}

}  // namespace bcosgpu
