/*
 * oracle.h -- CPU restatement of the FISCO-BCOS (v3.2.0) tx-admission / tx-root hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP engine in
 * fisco-bcos_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker / timed CPU baseline -- never as a product code path.
 *
 * Every function cites the reference file:line whose behaviour it restates.  The ECC parts
 * restate the third-party algorithms the reference delegates to (wedpr-crypto's libsecp256k1
 * recover, TASSL/OpenSSL sm2_do_verify): they are absent from /root/reference, so their
 * behaviour is pinned by the reference's own KATs (tests/golden/) and cross-checked here against
 * an independent OpenSSL 1.1.1 EC implementation (oracle/xcheck_openssl.c).
 */
#ifndef BCOS_ORACLE_H
#define BCOS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_KECCAK256 = 0, ORACLE_SM3 = 1 };
enum { ORACLE_SUITE_SECP256K1 = 0, ORACLE_SUITE_SM2 = 1 };

/* a1: OpenSSLHasher<Keccak256> (bcos-crypto/bcos-crypto/hasher/OpenSSLHasher.h:22-143, pad 0x01 :51-80) */
void oracle_keccak256(const uint8_t* in, size_t len, uint8_t out[32]);
/* a2: OpenSSLHasher<SM3> (OpenSSLHasher.h:113-116; hash/SM3.h:29-50) */
void oracle_sm3(const uint8_t* in, size_t len, uint8_t out[32]);
void oracle_hash(int hasher, const uint8_t* in, size_t len, uint8_t out[32]);
/* batch over a flat buffer: message i = data[offsets[i] .. offsets[i+1]) */
void oracle_hash_batch(int hasher, const uint8_t* data, const uint64_t* offsets, size_t n,
                       uint8_t* out32, int nthreads);

/* a9: Merkle<Hasher,width>::generateMerkle (bcos-crypto/bcos-crypto/merkle/Merkle.h:170-208).
 * Returns 0 on success, -1 for empty input (the reference throws std::invalid_argument).
 * levels (nullable) receives oracle_merkle_size(n,width) 32-byte entries in the reference's order:
 * per level a count record (uint32 big-endian in bytes 0..3, rest zero) followed by the nodes. */
int oracle_merkle(int hasher, int width, const uint8_t* leaves, size_t n, uint8_t root[32],
                  uint8_t* levels, int nthreads);
size_t oracle_merkle_size(size_t n, int width); /* Merkle.h:224-236 getMerkleSize */
/* a11: protocol::calculateMerkleProofRoot (bcos-protocol/bcos-protocol/ParallelMerkleProof.cpp:32-69) */
void oracle_merkle_old(int hasher, const uint8_t* leaves, size_t n, uint8_t root[32]);

/* a5: wedpr_secp256k1_recover_public_key semantics (Secp256k1Crypto.cpp:79-93).
 * sig = r(32) || s(32) || v(1).  Returns 0 and writes pub = X||Y (64 B) on success, -1 on failure. */
int oracle_secp256k1_recover(const uint8_t hash[32], const uint8_t* sig, size_t siglen,
                             uint8_t pub[64]);
/* secp256k1 priv->pub (SignatureTest.cpp:53-63).  -1 if sk is 0 or >= n. */
int oracle_secp256k1_pubkey(const uint8_t sk[32], uint8_t pub[64]);
/* libsecp256k1 sign_recoverable semantics (low-S, recid adjusted) with an explicit nonce k. */
int oracle_secp256k1_sign(const uint8_t sk[32], const uint8_t hash[32], const uint8_t k[32],
                          uint8_t sig[65]);
/* secp256k1Verify (Secp256k1Crypto.cpp:51-63) semantics: low-S required (libsecp256k1 verify). */
int oracle_secp256k1_verify(const uint8_t pub[64], const uint8_t hash[32], const uint8_t* sig,
                            size_t siglen);

/* a6: SM2Crypto::recover -> verify -> fast_sm2_verify (SM2Crypto.cpp:66-92, fast_sm2.cpp:139-227).
 * sig = r(32) || s(32) || pub(64).  Returns 0 if the signature verifies (pub written when non-null). */
int oracle_sm2_recover(const uint8_t hash[32], const uint8_t* sig, size_t siglen, uint8_t pub[64]);
int oracle_sm2_pubkey(const uint8_t sk[32], uint8_t pub[64]);
/* SM2 sign with explicit nonce k; writes r||s||pub (128 B). */
int oracle_sm2_sign(const uint8_t sk[32], const uint8_t hash[32], const uint8_t k[32],
                    uint8_t sig[128]);
/* Z_A for the reference's fixed user ID "1234567812345678" (fast_sm2.cpp:34) */
void oracle_sm2_za(const uint8_t pub[64], uint8_t za[32]);

/* a4 + a7 + a12: Transaction::verify (bcos-framework/.../protocol/Transaction.h:68-82) over a batch.
 * preimage i = pre[pre_off[i]..pre_off[i+1]) (TarsHashable.h:16-41), sig i = sig[sig_off[i]..].
 * Writes txhash32, sender20 (right160(H(pub)), KeyPair.h:30-33) and status (0 ok, 1 InvalidSignature). */
void oracle_tx_verify_batch(int suite, const uint8_t* pre, const uint64_t* pre_off,
                            const uint8_t* sig, const uint64_t* sig_off, size_t n,
                            uint8_t* txhash32, uint8_t* sender20, uint8_t* status, int nthreads);

/* raw batch recover/verify (for the CPU baseline) */
void oracle_secp256k1_recover_batch(const uint8_t* hash32, const uint8_t* sig65, size_t n,
                                    uint8_t* pub64, uint8_t* ok, int nthreads);
void oracle_sm2_verify_batch(const uint8_t* hash32, const uint8_t* sig128, size_t n, uint8_t* ok,
                             int nthreads);

#ifdef __cplusplus
}
#endif
#endif
