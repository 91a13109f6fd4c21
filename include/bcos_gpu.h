/*
 * bcos_gpu.h -- C ABI of the MI355X batch-verification engine for FISCO-BCOS's tx-admission and
 * block-check hot path (libbcosgpu.so).
 *
 * Drop-in boundary.  The reference reaches this path through
 *   - bcos::crypto::SignatureCrypto::recover / verify   bcos-crypto/bcos-crypto/interfaces/crypto/Signature.h:40-58
 *   - bcos::crypto::Hash::hash                          bcos-crypto/bcos-crypto/interfaces/crypto/Hash.h:44
 *   - bcos::crypto::merkle::Merkle<H,width>             bcos-crypto/bcos-crypto/merkle/Merkle.h:170-208
 * and, one level down, the wedpr / TASSL C ABI those classes bind (int8 return code, caller-owned
 * buffers): wedpr_secp256k1_recover_public_key (Secp256k1Crypto.cpp:79-93), wedpr_secp256k1_verify
 * (:51-63), fast_sm2_verify / wedpr_sm2_verify (fastsm2/fast_sm2.h:31-40, sm2/SM2Crypto.h:60-66).
 * This header exports (a) batch entry points -- what the batch sites TransactionSync::importDownloadedTxs
 * (bcos-txpool/bcos-txpool/sync/TransactionSync.cpp:516-548) and BlockImpl::calculateTransactionRoot
 * (bcos-tars-protocol/bcos-tars-protocol/protocol/BlockImpl.h:111-154) are rewired to -- and
 * (b) single-call shims with the exact wedpr signatures, so SignatureCrypto implementations can be
 * swapped without touching their callers.  include/bcos_gpu.hpp wraps (a) in the reference's C++
 * interface shapes; INTEGRATION.md shows the binding.
 *
 * Conventions: all functions return 0 on success and a negative BCOSGPU_E_* code on an API error
 * (never throw across the ABI); per-item crypto verdicts are written to caller-allocated ok[] /
 * status[] arrays (1 = valid / 0 = InvalidSignature for ok[]; 0 = ok, 1 = InvalidSignature for status[]).
 * Byte layouts are the reference's: 32-byte big-endian scalars and digests, 64-byte X||Y public keys
 * without the 0x04 prefix (Secp256k1KeyPair.h:29, SM2KeyPair.h:31), secp256k1 signatures r||s||v
 * (65 B, v = recovery id 0..3, SignatureDataWithV.h:43-61), SM2 signatures r||s||pub (128 B,
 * SignatureDataWithPub.h:55-64).  Functions are thread-safe.
 *
 * *_dev functions take DEVICE pointers and a hipStream_t (as void*; NULL = the legacy default
 * stream) and are stream-ordered: nothing is synchronised, nothing is allocated per call except the
 * engine's grow-only workspaces.  Device output pointers must be 4-byte aligned.  The other
 * functions take HOST pointers and return after the results are copied back.
 */
#ifndef BCOS_GPU_H
#define BCOS_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCOSGPU_VERSION 1

/* error codes */
#define BCOSGPU_OK 0
#define BCOSGPU_E_ARG (-1)    /* invalid argument (size, width, null pointer) */
#define BCOSGPU_E_HIP (-2)    /* HIP runtime error (see bcosgpu_last_error) */
#define BCOSGPU_E_NODEV (-3)  /* no usable gfx950 device */
#define BCOSGPU_E_EMPTY (-4)  /* empty Merkle input: the reference throws std::invalid_argument (Merkle.h:172-175) */

/* hashers (Hash implementations: hash/Keccak256.h, hash/SM3.h) */
#define BCOSGPU_KECCAK256 0
#define BCOSGPU_SM3 1
/* signature suites (libinitializer/ProtocolInitializer.cpp:102-124) */
#define BCOSGPU_SUITE_SECP256K1 0 /* Keccak256 + Secp256k1Crypto */
#define BCOSGPU_SUITE_SM2 1       /* SM3 + (Fast)SM2Crypto */
/* Merkle variants */
#define BCOSGPU_MERKLE_NEW 0 /* Merkle<H,width>::generateMerkle (Merkle.h:170-208) */
#define BCOSGPU_MERKLE_OLD 1 /* calculateMerkleProofRoot, width 16 (ParallelMerkleProof.cpp:32-69) */
#define BCOSGPU_MERKLE_NEW_BYTES 2 /* NEW, with `levels` in the vector<bytes> layout (bcosgpu_merkle_bytes_size) */

int bcosgpu_version(void);
/* Number of visible HIP devices (0 when none). */
int bcosgpu_device_count(void);
/* Select the calling thread's device and build its constant tables (idempotent). */
int bcosgpu_init(int device);
/* Same, with flags: BCOSGPU_INIT_SMALL_TABLES skips the two 64 MiB 16-bit comb tables (the kernels
 * then use the 512 KiB 8-bit ones, as they also do when the 64 MiB allocation fails).  Flags only
 * matter at a device's first initialisation. */
#define BCOSGPU_INIT_SMALL_TABLES 1
int bcosgpu_init_ex(int device, int flags);
/* Kernel selection for the tx-verify batch (tuning / tests; the default is chosen by batch size and
 * read once from BCOSGPU_TXV_SPLIT / _OCC / _COOP and BCOSGPU_K1_F26 at the first init, never per launch):
 * split -1 by size (secp256k1 batches <= 2^15 run the small-batch kernels), 0 never, 1 always;
 * occupancy 0 by size (2 waves/SIMD for n >= 2^17), 1 or 2 forced; coop (secp256k1 small batches)
 * 3 the row kernels (one signature per workgroup on row-spread field elements, ecc_row.hip: recovery,
 * and known-key verify through bcosgpu_verify_batch*), 2 lane-trio (default; needs field 1; with split -1
 * the automatic choice among row, lane-trio, pair and one-lane kernels by rounds x latency),
 * 1 cooperative-pair, 0 split (SM2: 3 the SM2 row kernel sm2_verify_row_kernel, 2 lane-trio, 1 pair
 * kernel, 0 the one-lane kernel);
 * field (secp256k1 throughput kernels) 1 the 10 x 26-bit point arithmetic (default), 0 the 8 x 32-bit
 * one, -1 unchanged.  Every variant returns identical results. */
int bcosgpu_set_tx_kernel_policy(int split, int occupancy, int coop, int field);
/* Last error message of the calling thread. */
const char* bcosgpu_last_error(void);
/* Bytes of the reference's Merkle output vector, in 32-byte entries (Merkle.h:224-236 getMerkleSize). */
uint64_t bcosgpu_merkle_size(uint64_t n, int width);

/* ---------------------------------------------------------------- hashing (Hash::hash, batched) */
/* message i = data[offsets[i] .. offsets[i+1]), n+1 offsets; out32 = n x 32-byte digests */
int bcosgpu_hash_batch(int hasher, const uint8_t* data, const uint64_t* offsets, size_t n,
                       uint8_t* out32);
int bcosgpu_keccak256_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32);
int bcosgpu_sm3_batch(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32);
int bcosgpu_hash_batch_dev(int hasher, const uint8_t* d_data, const uint64_t* d_offsets, size_t n,
                           uint8_t* d_out32, void* stream);

/* ---------------------------------------------------------------- Merkle (Merkle<H,width>) */
/* root32 receives the root; levels (nullable) receives bcosgpu_merkle_size(n,width) x 32 bytes laid
 * out as the reference's output vector: per level a count record (uint32 big-endian in bytes 0..3,
 * zero elsewhere) followed by the level's nodes; for n == 1 the single leaf.  variant OLD ignores
 * width (always 16) and levels; n == 0 returns H("") for OLD and BCOSGPU_E_EMPTY for NEW.
 * Variant NEW_BYTES: as NEW, with levels in the packed vector<bytes> layout (below). */
int bcosgpu_merkle_root(int hasher, int width, int variant, const uint8_t* leaves32, size_t n,
                        uint8_t* root32, uint8_t* levels);
/* d_tree must hold bcosgpu_merkle_size(n,width) x 32 bytes (>= 32 for n == 1). */
int bcosgpu_merkle_root_dev(int hasher, int width, const uint8_t* d_leaves32, size_t n,
                            uint8_t* d_tree, uint8_t* d_root32, void* stream);
/* The stored-tree layout of BlockImpl (m_inner->transactionsMerkle, a vector<vector<char>>,
 * BlockImpl.h:136) and merkleBench (vector<bytes>, merkleBench.cpp:53-56): generateMerkle into a
 * vector of byte buffers leaves each count record a 4-byte entry (setNumberToHash -> resizeTo(out, 4),
 * Merkle.h:213-217, concepts/bcos-concepts/Basic.h:50-61) and each node a 32-byte one.  Packed: the
 * entries back to back, count record (BE u32, 4 bytes) then that level's nodes (32 bytes each);
 * bcosgpu_merkle_bytes_size(n, width) bytes (32 for n == 1).  The 32-byte-entry layout above is the
 * one of fixed-size HashType vectors (Ledger proofs, LedgerTypeDef.h:27).
 * bcosgpu_merkle_tree_bytes_dev converts an output vector d_tree (of bcosgpu_merkle_root_dev for the
 * same n, width) into that layout at d_out (4-byte aligned, not overlapping d_tree);
 * bcosgpu_merkle_root(..., BCOSGPU_MERKLE_NEW_BYTES, ..., levels) returns it directly. */
uint64_t bcosgpu_merkle_bytes_size(uint64_t n, int width);
int bcosgpu_merkle_tree_bytes_dev(int width, const uint8_t* d_tree, size_t n, uint8_t* d_out, void* stream);

/* Multi-GPU tx root: compute `levels` levels of the reference tree over one shard of leaves.  The
 * shard's first global leaf index must be a multiple of width^levels; then its ceil(n / width^levels)
 * output nodes are exactly the reference's level-`levels` nodes for that range, and the root over the
 * concatenated frontiers of all shards (bcosgpu_merkle_root*) equals the single-device root.
 * d_work >= 64 * ceil(n / width) bytes; d_frontier receives ceil(n / width^levels) x 32 bytes. */
int bcosgpu_merkle_frontier_dev(int hasher, int width, const uint8_t* d_leaves32, size_t n, int levels,
                                uint8_t* d_work, uint8_t* d_frontier, void* stream);

/* Many blocks' roots in one call: BlockImpl::calculateTransactionRoot / calculateReceiptRoot
 * (bcos-tars-protocol/.../protocol/BlockImpl.h:111-183) for a batch of blocks, e.g. PBFT/sync replay.
 * Block b's leaves are entries [block_off[b], block_off[b+1]) of leaves32 (block_off: HOST array of
 * nblocks + 1 non-decreasing entry indices; leaves32 points at entry block_off[0]).  roots32[b] =
 * Merkle<H,width> root of block b; an empty block yields the zero hash (BlockImpl.h:114-119).
 * d_work >= bcosgpu_merkle_roots_work_size(block_off[nblocks] - block_off[0], nblocks, width) bytes. */
uint64_t bcosgpu_merkle_roots_work_size(uint64_t total_leaves, size_t nblocks, int width);
int bcosgpu_merkle_roots_batch(int hasher, int width, const uint8_t* leaves32, const uint64_t* block_off,
                               size_t nblocks, uint8_t* roots32);
int bcosgpu_merkle_roots_batch_dev(int hasher, int width, const uint8_t* d_leaves32, const uint64_t* block_off,
                                   size_t nblocks, uint8_t* d_work, uint8_t* d_roots32, void* stream);

/* Merkle proofs (Merkle<H,width>::generateMerkleProof / verifyMerkleProof, Merkle.h:45-168; callers
 * Ledger::getTransactionProof and the RPC proof queries).  A proof is a sequence of 32-byte entries:
 * per level below the root a count record (BE u32 in bytes 0..3) and the <= width nodes of the group
 * that contains the node (for a 1-leaf tree: the single leaf).  Proofs are written at a fixed stride
 * of bcosgpu_merkle_proof_stride(n, width) entries; proof_len[q] = entries used.
 * Index >= n is BCOSGPU_E_ARG ("Out of range!", Merkle.h:124-127).  Verification: ok[q] = 1 / 0, or
 * 2 for an empty proof (the reference throws std::invalid_argument{"Empty input proof!"}).  Roots: one
 * per proof (per_proof_root = 1) or one shared root (0). */
uint64_t bcosgpu_merkle_proof_stride(uint64_t n, int width);
int bcosgpu_merkle_proofs(int hasher, int width, const uint8_t* leaves32, size_t n, const uint64_t* index, size_t m,
                          uint8_t* proofs, uint32_t* proof_len);
/* d_tree = the output vector of bcosgpu_merkle_root_dev for the same leaves and width */
int bcosgpu_merkle_proofs_dev(int width, const uint8_t* d_leaves32, size_t n, const uint8_t* d_tree,
                              const uint64_t* d_index, size_t m, uint8_t* d_proofs, uint32_t* d_proof_len, void* stream);
int bcosgpu_merkle_verify_proofs(int hasher, const uint8_t* proofs, uint64_t stride, const uint32_t* proof_len,
                                 const uint8_t* hashes32, const uint8_t* roots32, int per_proof_root, size_t m,
                                 uint8_t* ok);
int bcosgpu_merkle_verify_proofs_dev(int hasher, const uint8_t* d_proofs, uint64_t stride, const uint32_t* d_proof_len,
                                     const uint8_t* d_hashes32, const uint8_t* d_roots32, int per_proof_root, size_t m,
                                     uint8_t* d_ok, void* stream);

/* ---------------------------------------------------------------- signatures (SignatureCrypto, batched) */
/* The host-pointer signature calls below (batched, single and the wedpr shims) are jobs of a
 * per-device queue: concurrent callers are coalesced into shared launches, each batch taking the
 * kernel the batch size calls for (the lane-trio / pair kernels for small batches, the one-lane kernel
 * at occupancy 1 or 2 for large ones; see bcosgpu_set_tx_kernel_policy).  Results are per call.
 * secp256k1 public-key recovery (Secp256k1Crypto::recover, Secp256k1Crypto.h:57-60).
 * pub64 / addr20 nullable; addr20 = right160(Keccak256(pub)) (calculateAddress, KeyPair.h:30-33). */
int bcosgpu_secp256k1_recover_batch(const uint8_t* hash32, const uint8_t* sig65, size_t n,
                                    uint8_t* pub64, uint8_t* addr20, uint8_t* ok);
int bcosgpu_secp256k1_recover_batch_dev(const uint8_t* d_hash32, const uint8_t* d_sig65, size_t n,
                                        uint8_t* d_pub64, uint8_t* d_addr20, uint8_t* d_ok,
                                        void* stream);
/* SM2 verify with the embedded public key (SM2Crypto::recover, SM2Crypto.cpp:81-92).
 * addr20 = right160(SM3(pub)), nullable. */
int bcosgpu_sm2_verify_batch(const uint8_t* hash32, const uint8_t* sig128, size_t n,
                             uint8_t* addr20, uint8_t* ok);
int bcosgpu_sm2_verify_batch_dev(const uint8_t* d_hash32, const uint8_t* d_sig128, size_t n,
                                 uint8_t* d_addr20, uint8_t* d_ok, void* stream);
/* Key derivation + deterministic signing (SignatureCrypto::createKeyPair / sign), used to build
 * synthetic signed batches on the device.  TEST / BENCHMARK USE ONLY: not constant-time (the comb
 * gather addresses depend on key and nonce bits) -- the reference signs on the host.  Nonce k = H(sk || hash) mod n (H = Keccak256 for
 * secp256k1, SM3 for SM2); sig65 = r||s||v (low-S, libsecp256k1 convention), sig128 = r||s||pub.
 * ok[i] = 0 when sk is out of range or the nonce is degenerate. */
int bcosgpu_secp256k1_sign_batch_dev(const uint8_t* d_sk32, const uint8_t* d_hash32, size_t n,
                                     uint8_t* d_pub64, uint8_t* d_sig65, uint8_t* d_ok, void* stream);
int bcosgpu_sm2_sign_batch_dev(const uint8_t* d_sk32, const uint8_t* d_hash32, size_t n,
                               uint8_t* d_sig128, uint8_t* d_ok, void* stream);

/* SignatureCrypto::verify(pub, hash, sig) with a KNOWN key (Signature.h:40-46), batched -- the sealer
 * signature checks BlockValidator::checkSignatureList (bcos-pbft/.../engine/BlockValidator.cpp:141-182)
 * and PBFTCacheProcessor::checkPrecommitWeight (.../cache/PBFTCacheProcessor.cpp:795-821).
 *   secp256k1: secp256k1Verify -> wedpr_secp256k1_verify (Secp256k1Crypto.cpp:51-63), libsecp256k1
 *              secp256k1_ecdsa_verify semantics (low-S required, pub on the curve);
 *   SM2:       SM2Crypto::verify (SM2Crypto.cpp:66-79) -> sm2_do_verify against the given key.
 * Item i: pub64 + 64 i, hash32 + 32 i, signature sig + sig_stride i (stride >= 64: 65 for r||s||v,
 * 128 for r||s||pub; only bytes 0..63 = r||s are read).  ok[i] = 1 iff the signature verifies. */
int bcosgpu_verify_batch(int suite, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig,
                         size_t sig_stride, size_t n, uint8_t* ok);
int bcosgpu_verify_batch_dev(int suite, const uint8_t* d_pub64, const uint8_t* d_hash32, const uint8_t* d_sig,
                             size_t sig_stride, size_t n, uint8_t* d_ok, void* stream);

/* Registered keys: the sealer path.  BlockValidator::checkSignatureList and
 * PBFTCacheProcessor::checkPrecommitWeight verify against the consensus node list's keys -- a small
 * set known in advance (ConsensusNode list; PBFTConfig).  A registered key gets an 8-bit comb table of
 * its multiples in HBM (512 KiB, built once), so verifying against it needs table lookups and ~7 point
 * additions instead of a variable-base multiplication (~10x shorter per signature; same verdicts).
 *   bcosgpu_register_keys: tables for n keys (pub64 + 64 i) of `suite` on `device`; slots[i] = the key's
 *     slot id (opaque, >= 0), or -1 when the cache is full (BCOSGPU_KEY_CACHE keys per device and suite,
 *     default 256).  Returns the number of keys cached (< 0 on error).  Registering a cached key is a lookup.
 *   Host-pointer verify calls (bcosgpu_verify_batch, bcosgpu_secp256k1_verify, bcosgpu_sm2_verify, the
 *     device-set batches, SM2 recover) take the registered-key kernel when every key of the coalesced
 *     batch is cached.  A key NAMED (pub64 given: the sealer path) in BCOSGPU_KEY_PROMOTE (default 3;
 *     0 = never) verify calls is cached automatically -- counted once per call, at most 16 new tables per
 *     call, in at most half the capacity (the other half is kept for registrations); SM2 recover
 *     (admission, the sender's embedded key) only looks keys up.
 *   bcosgpu_verify_keyed_batch_dev: ok[i] = verify(key of slot id d_slots[i], d_hash32 + 32 i, d_sig +
 *     sig_stride i) on the calling thread's device, stream-ordered; an id that names no registered key
 *     fails (ok = 0) -- including every id handed out before a bcosgpu_clear_keys: ids carry the cache
 *     generation, so an old id never verifies against a key registered later in the same index.
 *   bcosgpu_key_cache_info: out5 = {keys cached, capacity, verified on the keyed path, verified
 *     elsewhere, tables built}.  bcosgpu_clear_keys: drains the device, then forgets every key (a
 *     consensus membership change); later registrations get new ids (a coalesced batch that looked its
 *     keys up before the clear runs again on the generic kernels). */
int bcosgpu_register_keys(int device, int suite, const uint8_t* pub64, size_t n, int32_t* slots);
int bcosgpu_verify_keyed_batch_dev(int suite, const int32_t* d_slots, const uint8_t* d_hash32, const uint8_t* d_sig,
                                   size_t sig_stride, size_t n, uint8_t* d_ok, void* stream);
int bcosgpu_key_cache_info(int device, int suite, int64_t* out5);
int bcosgpu_clear_keys(int device, int suite);

/* EVM ecRecover precompile (bcos-executor/src/vm/Precompiled.cpp:443-482), batched.  Input i =
 * in128 + 128 i = hash(32) || v(32) || r(32) || s(32); the recovery id is (uint8_t)(in[63] - 27).
 * On success out32 = 12 zero bytes || right160(Keccak256(pub)) and ok = 1; on failure the precompile
 * returns an empty output: ok = 0 (out32 zero).  d_in128 must be 16-byte aligned. */
int bcosgpu_ecrecover_batch(const uint8_t* in128, size_t n, uint8_t* out32, uint8_t* ok);
int bcosgpu_ecrecover_batch_dev(const uint8_t* d_in128, size_t n, uint8_t* d_out32, uint8_t* d_ok, void* stream);

/* ---------------------------------------------------------------- whole-tx admission (Transaction::verify, batched) */
/* Transaction::verify (bcos-framework/.../protocol/Transaction.h:68-82) for n transactions:
 * txhash = H(preimage) (TarsHashable.h:16-41), pub = recover(txhash, sig), sender = right160(H(pub)).
 * preimage i = pre[pre_off[i] .. pre_off[i+1]); signature i = sig[sig_off[i] .. sig_off[i+1]).
 * status[i] = 0 (ok) or 1 (TransactionStatus::InvalidSignature); sender20 zero when invalid. */
int bcosgpu_tx_verify_batch(int suite, const uint8_t* pre, const uint64_t* pre_off,
                            const uint8_t* sig, const uint64_t* sig_off, size_t n,
                            uint8_t* txhash32, uint8_t* sender20, uint8_t* status);
int bcosgpu_tx_verify_batch_dev(int suite, const uint8_t* d_pre, const uint64_t* d_pre_off,
                                const uint8_t* d_sig, const uint64_t* d_sig_off, size_t n,
                                uint8_t* d_txhash32, uint8_t* d_sender20, uint8_t* d_status,
                                void* stream);

/* ---------------------------------------------------------------- Tars-encoded transactions */
/* Batched TransactionFactoryImpl::createTransaction(txData, checkSig, checkHash)
 * (bcos-tars-protocol/bcos-tars-protocol/protocol/TransactionFactoryImpl.h:46-85), decode included:
 * decode n Tars-encoded bcostars::Transaction (TransactionImpl.cpp:38-41 -> TarsSerializable.h:28-35, the
 * tarscpp wire format), recompute the tx hash and, when check_sig, recover / verify the signature and
 * derive the sender (sender = 0 otherwise).  Callers: JsonRpcImpl_2_0.cpp:443-444 (sendTransaction,
 * checkSig false, checkHash true), TxPool.cpp:96 (pushed txs, checkSig false).
 * Encoded tx i = enc[enc_off[i] .. enc_off[i+1]).  status[i]: 0 ok, 1 InvalidSignature (verify throws),
 * 2 the decode throws, 3 check_hash != 0 and a non-empty dataHash differs from the recomputed hash. */
int bcosgpu_tars_tx_verify_batch(int suite, const uint8_t* enc, const uint64_t* enc_off, size_t n, int check_sig,
                                 int check_hash, uint8_t* txhash32, uint8_t* sender20, uint8_t* status);
/* Work buffer for the device entry points below: >= bcosgpu_tars_decode_work_size(n) bytes. */
uint64_t bcosgpu_tars_decode_work_size(size_t n);
/* Device decode only: writes the packed preimages / signatures in the layout bcosgpu_tx_verify_batch_dev
 * takes.  d_pre >= enc bytes + 12 n, d_sig >= enc bytes, d_pre_off / d_sig_off n + 1 entries,
 * d_dec_status n bytes (0 / 2; may be null). */
int bcosgpu_tars_tx_decode_dev(const uint8_t* d_enc, const uint64_t* d_enc_off, size_t n, uint8_t* d_pre,
                               uint64_t* d_pre_off, uint8_t* d_sig, uint64_t* d_sig_off, uint8_t* d_dec_status,
                               void* d_work, uint64_t work_bytes, void* stream);
/* Device decode + verify, stream-ordered (the buffers as for bcosgpu_tars_tx_decode_dev). */
int bcosgpu_tars_tx_verify_batch_dev(int suite, const uint8_t* d_enc, const uint64_t* d_enc_off, size_t n,
                                     int check_sig, int check_hash, uint8_t* d_pre, uint64_t* d_pre_off, uint8_t* d_sig,
                                     uint64_t* d_sig_off, void* d_work, uint64_t work_bytes, uint8_t* d_txhash32,
                                     uint8_t* d_sender20, uint8_t* d_status, void* stream);

/* ---------------------------------------------------------------- host-side preimage packer */
/* A view of bcostars::TransactionData (bcos-tars-protocol/.../tars/Transaction.tars:2-11): pointers
 * into the caller's decoded transaction, nothing is copied until packing. */
typedef struct {
    int32_t version;
    const char* chain_id;  size_t chain_id_len;
    const char* group_id;  size_t group_id_len;
    int64_t block_limit;
    const char* nonce;     size_t nonce_len;
    const char* to;        size_t to_len;
    const uint8_t* input;  size_t input_len;
    const char* abi;       size_t abi_len;
} bcosgpu_TransactionData;
/* Total preimage bytes of n transactions. */
uint64_t bcosgpu_tx_preimage_size(const bcosgpu_TransactionData* txs, size_t n);
/* Packs the tx-hash preimages impl_calculate<Hasher>(Transaction) hashes (TarsHashable.h:16-41:
 * be32(version) || chainID || groupID || be64(blockLimit) || nonce || to || input || abi) back to
 * back into out (cap bytes) and writes offsets[n+1] -- the SoA layout bcosgpu_tx_verify_batch* take.
 * Host only (no device needed); multithreaded for large batches.  BCOSGPU_E_ARG if cap is too small. */
int bcosgpu_pack_tx_preimages(const bcosgpu_TransactionData* txs, size_t n, uint8_t* out, uint64_t cap,
                              uint64_t* offsets);

/* ---------------------------------------------------------------- receipts (calculateReceiptRoot) */
/* Views of bcostars::LogEntry / TransactionReceiptData / TransactionReceipt.dataHash
 * (bcos-tars-protocol/bcos-tars-protocol/tars/TransactionReceipt.tars:2-23): pointers into the caller's
 * decoded receipt.  topic is vector<vector<byte>>: ntopics byte strings. */
typedef struct { const uint8_t* data; size_t len; } bcosgpu_Bytes;
typedef struct {
    const char* address;   size_t address_len;
    const bcosgpu_Bytes* topics; size_t ntopics;
    const uint8_t* data;   size_t data_len;
} bcosgpu_LogEntry;
typedef struct {
    int32_t version;
    const char* gas_used;          size_t gas_used_len;
    const char* contract_address;  size_t contract_address_len;
    int32_t status;
    const uint8_t* output;         size_t output_len;
    const bcosgpu_LogEntry* logs;  size_t nlogs;
    int64_t block_number;
    /* TransactionReceipt.dataHash: when non-empty it IS the receipt hash (TarsHashable.h:47-51) and the
     * fields above are not read.  At most 32 bytes (the reference's assignTo into a 32-byte hash throws
     * NoEnoughSpace beyond that); a shorter one fills the leading bytes, the rest are zero here (the
     * reference leaves them uninitialised, BlockImpl.h:171). */
    const uint8_t* data_hash;      size_t data_hash_len;
} bcosgpu_TransactionReceiptData;
/* Total preimage bytes of n receipts (0 for a receipt with a dataHash). */
uint64_t bcosgpu_receipt_preimage_size(const bcosgpu_TransactionReceiptData* receipts, size_t n);
/* Packs the receipt-hash preimages impl_calculate<Hasher>(TransactionReceipt) hashes
 * (TarsHashable.h:54-73: be32(version) || gasUsed || contractAddress || be32(status) || output ||
 * per log (address || topic_0 .. topic_k || data) || be64(blockNumber)) back to back into out (cap bytes)
 * and writes offsets[n+1]; a receipt with a dataHash gets an empty preimage.  Host only, multithreaded
 * for large batches.  BCOSGPU_E_ARG if cap is too small, a field pointer is null with a non-zero length,
 * or a dataHash is longer than 32 bytes. */
int bcosgpu_pack_receipt_preimages(const bcosgpu_TransactionReceiptData* receipts, size_t n, uint8_t* out,
                                   uint64_t cap, uint64_t* offsets);
/* hashes32[i] = receipt i's dataHash for every receipt that has one (host only; the step after hashing
 * the packed preimages). */
void bcosgpu_apply_receipt_data_hashes(const bcosgpu_TransactionReceiptData* receipts, size_t n, uint8_t* hashes32);
/* BlockImpl::calculateReceiptRoot (bcos-tars-protocol/.../protocol/BlockImpl.h:156-183) for nblocks blocks
 * in one call: block b's receipts are receipts[block_off[b] .. block_off[b+1]) (HOST array, block_off[0] =
 * 0); every receipt hashed on the GPU with `hasher` (impl_calculate, dataHash short-circuit), then
 * roots32 + 32 b = Merkle<H, 2> root of block b's receipt hashes (zero hash for a block without
 * receipts, BlockImpl.h:159-163).  hashes32 (nullable) receives the block_off[nblocks] receipt hashes. */
int bcosgpu_receipt_roots(int hasher, const bcosgpu_TransactionReceiptData* receipts, const uint64_t* block_off,
                          size_t nblocks, uint8_t* roots32, uint8_t* hashes32);

/* ---------------------------------------------------------------- single calls on an explicit device */
/* One signature per call, for the reference's per-transaction call sites: TxPool's submitter threads
 * (TxPool.h:48-49) -> TxValidator::verify (TxValidator.cpp:56) -> Transaction::verify (Transaction.h:68-82)
 * -> SignatureCrypto::recover.  Concurrent calls on one device are coalesced into shared launches (one
 * H2D copy, one kernel, one D2H copy per batch; up to 4 batches in flight per device).  `device` is
 * initialised on first use; the calling thread's current device is left unchanged.
 * Return 1 = valid, 0 = invalid signature (the reference throws InvalidSignature / returns false),
 * < 0 = engine error (BCOSGPU_E_*, message in bcosgpu_last_error()). */
/* Secp256k1Crypto::recover (Secp256k1Crypto.cpp:79-93): sig = r||s||v, sig_len must be 65;
 * pub64 = X||Y (zero when invalid). */
int bcosgpu_secp256k1_recover(int device, const uint8_t* hash32, const uint8_t* sig, size_t sig_len, uint8_t* pub64);
/* secp256k1Verify -> wedpr_secp256k1_verify (Secp256k1Crypto.cpp:51-63): libsecp256k1 verify (low-S);
 * only sig[0..64) = r||s is read; sig_len < 64 is invalid. */
int bcosgpu_secp256k1_verify(int device, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig,
                             size_t sig_len);
/* SM2Crypto::verify (SM2Crypto.cpp:66-79) -> fast_sm2_verify: sig64 = r||s, with the given key. */
int bcosgpu_sm2_verify(int device, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig64);
/* Where the coalesced calls' time goes on `device` (diagnostics; counters since start or the last reset):
 * out10 = {batches, calls, signatures, queue ns (sum over calls: enqueued -> taken into a batch), leader ns
 * (sum over batches: staging and key lookup before the launch), GPU ns (launch -> results synchronised),
 * scatter ns (results copied to the callers), wake ns (sum over targeted wake-ups: notify -> running),
 * wake-ups, lock ns (sum over calls: waiting for the queue mutex)}; reset != 0 zeroes them. */
int bcosgpu_coalesce_stats(int device, uint64_t* out10, int reset);

/* ---------------------------------------------------------------- device sets (one process, several GPUs) */
/* A FISCO node is ONE process with one CryptoSuite (libinitializer/ProtocolInitializer.cpp:102-124) whose
 * batch sites run in-process (TransactionSync.cpp:516-548, BlockImpl.h:111-154); these entry points let
 * that process use all the GPUs of its node (SURVEY 8(b) "one context per GPU", 8(e)).  `devices` lists
 * ndev device indices (1 <= ndev <= 64); a batch is split by index into ndev contiguous shards, shard k
 * running on devices[k] on its own stream with its own buffers -- an index may repeat (two shards on one
 * GPU, distinct streams).  Results are identical to the single-device calls for every n.  Host pointers;
 * the calling thread's current device is left unchanged.  Test status: every entry point is checked
 * against the oracle on repeated-device lists ({0, 0}, {0, 0, 0}), including the cross-device peer-copy
 * gather (forced by BCOSGPU_MULTI_PEER=1); lists of distinct physical GPUs have not run on hardware yet.
 * Initialise every device of the set (tables, streams); idempotent. */
int bcosgpu_init_devices(const int* devices, int ndev);
/* The signature batches above, sharded over the set (each shard a coalesced job on its device). */
int bcosgpu_secp256k1_recover_batch_multi(const int* devices, int ndev, const uint8_t* hash32, const uint8_t* sig65,
                                          size_t n, uint8_t* pub64, uint8_t* addr20, uint8_t* ok);
int bcosgpu_sm2_verify_batch_multi(const int* devices, int ndev, const uint8_t* hash32, const uint8_t* sig128,
                                   size_t n, uint8_t* addr20, uint8_t* ok);
int bcosgpu_verify_batch_multi(const int* devices, int ndev, int suite, const uint8_t* pub64, const uint8_t* hash32,
                               const uint8_t* sig, size_t sig_stride, size_t n, uint8_t* ok);
/* bcosgpu_tx_verify_batch over the set: TransactionSync::importDownloadedTxs' verify loop
 * (TransactionSync.cpp:516-548) for a whole download on every GPU of the node. */
int bcosgpu_tx_verify_batch_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                                  const uint8_t* sig, const uint64_t* sig_off, size_t n, uint8_t* txhash32,
                                  uint8_t* sender20, uint8_t* status);
/* Block check in one call: bcosgpu_tx_verify_batch_multi plus the block's tx root
 * (BlockImpl::calculateTransactionRoot, BlockImpl.h:111-154: Merkle<H, width> over the tx hashes, H =
 * Keccak256 / SM3 by suite; zero hash for an empty block).  Shard starts are multiples of width^L, each
 * GPU reduces its shard's hashes to the reference tree's level-L nodes, the frontiers (a few KB) are
 * gathered on devices[0] with peer copies over xGMI, and the top levels run there. */
int bcosgpu_block_verify_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                               const uint8_t* sig, const uint64_t* sig_off, size_t n, int width, uint8_t* txhash32,
                               uint8_t* sender20, uint8_t* status, uint8_t* root32);
/* Many blocks in one call (a sync catch-up / replay of downloaded blocks, configs[4]): block b's txs are
 * [block_off[b], block_off[b+1]) (block_off[0] = 0, nblocks + 1 entries), every tx verified as
 * bcosgpu_tx_verify_batch does and roots32 + 32 b = block b's tx root (zero hash for an empty block).
 * Whole blocks go to the devices in contiguous ranges balanced by tx count; no exchange. */
int bcosgpu_blocks_verify_multi(const int* devices, int ndev, int suite, const uint8_t* pre, const uint64_t* pre_off,
                                const uint8_t* sig, const uint64_t* sig_off, const uint64_t* block_off, size_t nblocks,
                                int width, uint8_t* txhash32, uint8_t* sender20, uint8_t* status, uint8_t* roots32);
/* Merkle<H, width>::generateMerkle's root (Merkle.h:170-208) over the set, by the same frontier scheme;
 * n == 0 is BCOSGPU_E_EMPTY, n == 1 returns the leaf. */
int bcosgpu_merkle_root_multi(const int* devices, int ndev, int hasher, int width, const uint8_t* leaves32, size_t n,
                              uint8_t* root32);

/* ---------------------------------------------------------------- wedpr-ABI single-call shims */
/* Same layout as wedpr-crypto's CInputBuffer / COutputBuffer; on the calling thread's current device.
 * Return 0 (WEDPR_SUCCESS), -1 (WEDPR_ERROR: invalid input or signature) or
 * BCOSGPU_WEDPR_ENGINE_ERROR when the engine itself failed (no gfx950 device, HIP error; message in
 * bcosgpu_last_error()) -- a reference caller that only tests "!= WEDPR_SUCCESS" reads that as an
 * invalid signature, so the SignatureCrypto adapters (bcos_gpu_crypto.hpp) check for it and throw
 * SignException instead.
 * A reference translation unit that already has wedpr's types (<wedpr-crypto/WedprCrypto.h>) includes
 * bcos_gpu_wedpr.h instead, which declares these two symbols over CInputBuffer / COutputBuffer so they
 * bind to SM2Crypto::m_verifier (SM2Crypto.h:64-65) and to wedpr's call sites unchanged. */
#define BCOSGPU_WEDPR_ENGINE_ERROR (-2)
typedef struct { const char* data; uintptr_t len; } bcosgpu_CInputBuffer;
typedef struct { char* data; uintptr_t len; } bcosgpu_COutputBuffer;
#ifndef BCOSGPU_WEDPR_TYPES
/* wedpr_secp256k1_recover_public_key (Secp256k1Crypto.cpp:79-93) */
int8_t bcosgpu_wedpr_secp256k1_recover_public_key(const bcosgpu_CInputBuffer* hash,
                                                   const bcosgpu_CInputBuffer* sig,
                                                   bcosgpu_COutputBuffer* pub);
/* fast_sm2_verify / wedpr_sm2_verify (fast_sm2.cpp:139-227): sig = r||s (64 B), pub = 64 B */
int8_t bcosgpu_wedpr_sm2_verify(const bcosgpu_CInputBuffer* pub, const bcosgpu_CInputBuffer* hash,
                                 const bcosgpu_CInputBuffer* sig);
/* wedpr_secp256k1_verify (Secp256k1Crypto.cpp:51-63): libsecp256k1 verify semantics (low-S) */
int8_t bcosgpu_wedpr_secp256k1_verify(const bcosgpu_CInputBuffer* pub, const bcosgpu_CInputBuffer* hash,
                                      const bcosgpu_CInputBuffer* sig);
#endif

#ifdef __cplusplus
}
#endif
#endif
