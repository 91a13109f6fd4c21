// engine.h -- internal launcher declarations shared by the kernel TUs and the C ABI (api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <string>
#include <vector>
#include "../../include/bcos_gpu.h"

namespace bcosgpu {

// compute units of the current device (cached per device)
inline int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}

// hash_kernels.hip
int launch_hash_batch(int hasher, const uint8_t* d_data, const uint64_t* d_off, uint64_t n,
                      uint8_t* d_out, hipStream_t st);
uint64_t merkle_size(uint64_t n, int width);
int launch_merkle(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                  uint8_t* d_root, hipStream_t st);
int launch_merkle_levels(int hasher, int width, const uint8_t* d_in, uint64_t n, int levels, uint8_t* d_work,
                         uint8_t* d_out, hipStream_t st);
uint64_t merkle_roots_work_bytes(uint64_t total_leaves, uint64_t nblocks, int width);
int launch_merkle_roots_batch(int hasher, int width, const uint8_t* d_leaves, const uint64_t* block_off,
                              uint64_t nblocks, uint8_t* d_work, uint8_t* d_roots, hipStream_t st);
uint64_t merkle_proof_stride(uint64_t n, int width);
int launch_merkle_proofs(int width, const uint8_t* d_leaves, uint64_t n, const uint8_t* d_tree, const uint64_t* d_index,
                         uint64_t m, uint8_t* d_proofs, uint32_t* d_len, hipStream_t st);
int launch_merkle_verify(int hasher, const uint8_t* d_proofs, uint64_t stride, const uint32_t* d_len,
                         const uint8_t* d_hashes, const uint8_t* d_roots, int root_stride, uint64_t m, uint8_t* d_ok,
                         hipStream_t st);
int launch_merkle_old(int hasher, const uint8_t* d_leaves, uint64_t n, uint8_t* d_scratch,
                      uint8_t* d_root, hipStream_t st);
uint64_t merkle_levels(uint64_t n, int width);
// the output vector -> the packed vector<bytes> layout (4-byte count records)
int launch_merkle_compact(const uint8_t* d_tree, uint64_t n, int width, uint8_t* d_out, hipStream_t st);

// ecc_tables.hip, ecc_sig.hip, ecc_txv.hip (the ECC kernels: tables, signing, verify / recover launchers)
int ecc_init_tables(int device, int small_tables);
void set_tx_kernel_policy(int split, int occ, int coop, int f26);
int launch_secp256k1_recover(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t sig_stride,
                             uint64_t n, uint8_t* d_pub, uint8_t* d_addr, uint8_t* d_ok,
                             hipStream_t st);
int launch_sm2_verify(const uint8_t* d_hash, const uint8_t* d_sig, uint32_t sig_stride, uint64_t n,
                      uint8_t* d_addr, uint8_t* d_ok, hipStream_t st);
int launch_secp256k1_sign(const uint8_t* d_sk, const uint8_t* d_hash, uint64_t n, uint8_t* d_pub,
                          uint8_t* d_sig, uint8_t* d_ok, hipStream_t st);
int launch_sm2_sign(const uint8_t* d_sk, const uint8_t* d_hash, uint64_t n, uint8_t* d_sig,
                    uint8_t* d_ok, hipStream_t st);
int launch_sig_verify(int suite, const uint8_t* d_pub, const uint8_t* d_hash, const uint8_t* d_sig, uint32_t stride,
                      uint64_t n, uint8_t* d_ok, hipStream_t st);
int launch_ecrecover(const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint8_t* d_ok, hipStream_t st);
int launch_tx_verify(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off,
                     const uint8_t* d_sig, const uint64_t* d_sig_off, uint64_t n,
                     uint8_t* d_txhash, uint8_t* d_sender, uint8_t* d_status, hipStream_t st);

// ecc_keyed.hip: verification against registered keys (per-key comb tables in HBM)
int keyed_slots(int suite, const uint8_t* pubs, size_t pub_stride, size_t n, int32_t* out, bool force, bool* all,
                hipStream_t st, uint64_t* gen = nullptr, bool promote = false);
uint64_t keyed_generation(int suite);  // of the current device's cache
int launch_sig_verify_keyed(int suite, const int32_t* d_slots, const uint8_t* d_hash, const uint8_t* d_sig,
                            uint32_t stride, uint64_t n, uint8_t* d_ok, uint8_t* d_addr, hipStream_t st);
int keyed_cache_info(int device, int suite, int64_t out[5]);
int keyed_clear(int device, int suite);

// coalesce.hip: the host-pointer signature calls as jobs of a per-device queue, coalesced into shared
// launches (see the file header).  coalesced_run blocks until the job's results are written.
enum SigJobKind { kSigJobRecoverK1 = 0, kSigJobVerifySM2 = 1, kSigJobVerifyK1 = 2, kSigJobKinds = 3 };
struct SigJob {
    int kind = 0;
    size_t n = 0;
    const uint8_t* hash32 = nullptr;  // n x 32
    const uint8_t* sig = nullptr;     // item i at sig + sig_stride * i: r||s||v (recover), r||s[||pub] (verify)
    size_t sig_stride = 0;
    const uint8_t* pub64 = nullptr;   // verify: the known keys (SM2: null = the key is sig[64..128))
    uint8_t* out_pub64 = nullptr;     // recover only, nullable
    uint8_t* out_addr20 = nullptr;    // recover / SM2 verify, nullable
    uint8_t* out_ok = nullptr;        // n bytes: 1 valid, 0 invalid
    int rc = 0;                       // filled in by the engine: 0 or BCOSGPU_E_*, with err
    std::string err;
    bool queued = false, woken = false;  // under the device queue's mutex
    uint64_t seq = 0;                    // arrival order in its device queue
    int64_t t_enq = 0;                   // steady-clock ns: queued (coalescer statistics)
    std::atomic<int64_t> t_notify{0};    // ... last notified
    std::atomic<uint32_t> wake{0};       // the owner's futex word: bit 0 woken to lead, bit 1 done (coalesce.hip)
    SigJob* next = nullptr;              // the device queue's lock-free arrival stack
};
int coalesced_run(int device, SigJob& job);
int coalesce_stats(int device, uint64_t* out, int n, int reset);

// api.hip internals the device-set entry points (multi.hip) share: the calling thread's error message,
// one-time device initialisation without changing the calling thread's device, a coalesced job
int api_set_err(int code, const std::string& msg);
int api_ready_device(int device);
int api_run_job(int device, SigJob& job);

// txpipe.hip: the host-pointer tx-verify batches as a chunked copy / compute pipeline (see the file header)
struct PipeBuf {  // grow-only device buffer
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes);
    template <class T> T* as() const { return static_cast<T*>(p); }
};
struct PipeHostBuf {  // grow-only pinned host buffer, mapped into the device's address space (hd)
    void* p = nullptr;
    void* hd = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes);
    template <class T> T* as() const { return static_cast<T*>(p); }
};
struct TxPipe {
    int device = -1;
    hipStream_t compute = nullptr, compute2 = nullptr, copy = nullptr;  // chunks alternate compute streams
    std::vector<hipEvent_t> ev;  // 2 per chunk: inputs landed, kernel done
    PipeBuf b[8];                // 0-4 the pipeline's (inputs, outputs); 5-7 free for a tail's work
    PipeHostBuf hin, host;       // input / output staging of small batches
};
// txs [lo, hi) of a host batch (the caller's indexing: offsets, outputs at row i for tx i)
struct HostTxRange {
    int suite = 0;
    const uint8_t* pre = nullptr;
    const uint64_t* pre_off = nullptr;
    const uint8_t* sig = nullptr;
    const uint64_t* sig_off = nullptr;
    uint64_t lo = 0, hi = 0;
    uint8_t* txhash32 = nullptr;
    uint8_t* sender20 = nullptr;
    uint8_t* status = nullptr;
    // shards of the same call with work on this range's device (txpipe.hip): alone (1), the pipeline
    // starts with a quarter-round head chunk and then takes whole rounds; shared, no head chunk (the other
    // shards' first chunks already fill the GPU beside it) and chunks of one round / share
    int share = 1;
};
// queued on p.compute after every chunk's kernel, before the last download: d_hash = the range's
// (hi - lo) x 32 tx hashes on the device
using PipeTail = std::function<int(TxPipe& p, const uint8_t* d_hash, std::string& msg)>;
TxPipe* tx_pipe_acquire(int device);  // nullptr on a HIP failure; the calling thread's device is kept
void tx_pipe_release(TxPipe* p);
uint64_t tx_pipe_chunk(uint64_t m, int share = 1);
// on the calling thread's current device == p.device; returns after every output is in host memory
int tx_pipeline(TxPipe& p, const HostTxRange& t, const PipeTail& tail, std::string& msg);

// tars_kernels.hip
uint64_t tars_decode_work_bytes(uint64_t n);
int launch_tars_tx_decode(const uint8_t* d_enc, const uint64_t* d_enc_off, uint64_t n, uint8_t* d_pre,
                          uint64_t* d_pre_off, uint8_t* d_sig, uint64_t* d_sig_off, uint8_t* d_dec_status,
                          void* d_work, uint64_t work_bytes, hipStream_t st);
// d_dec may be null: the decode status kept in d_work by launch_tars_tx_decode(d_dec_status = null)
int launch_tars_finish(const uint8_t* d_enc, const void* d_work, const uint8_t* d_dec, const uint8_t* d_txhash,
                       uint8_t* d_status, uint64_t n, int check_hash, hipStream_t st);

}  // namespace bcosgpu
