/*
 * batch.c -- multi-threaded batch drivers of the oracle (the CPU baseline).  TEST INFRASTRUCTURE ONLY.
 *
 * Mirrors the reference's batch site TransactionSync::importDownloadedTxs
 * (bcos-txpool/bcos-txpool/sync/TransactionSync.cpp:496-575: tbb::parallel_for over tx indices,
 * each calling Transaction::verify, bcos-framework/.../protocol/Transaction.h:68-82).
 */
#include "oracle.h"
#include "parallel.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct { oracle_range_fn fn; void* ctx; size_t lo, hi; } job;
static void* run_job(void* p)
{
    job* j = (job*)p;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}

void oracle_parallel_for(size_t n, int nthreads, oracle_range_fn fn, void* ctx)
{
    if (nthreads <= 1 || n < 2) { fn(ctx, 0, n); return; }
    if ((size_t)nthreads > n) nthreads = (int)n;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    job* jobs = (job*)malloc(sizeof(job) * (size_t)nthreads);
    for (int t = 0; t < nthreads; ++t) { /* contiguous shards */
        jobs[t].fn = fn; jobs[t].ctx = ctx;
        jobs[t].lo = n * (size_t)t / (size_t)nthreads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

typedef struct { int hasher; const uint8_t* data; const uint64_t* off; uint8_t* out; } hash_ctx;
static void hash_range(void* p, size_t lo, size_t hi)
{
    hash_ctx* c = (hash_ctx*)p;
    for (size_t i = lo; i < hi; ++i)
        oracle_hash(c->hasher, c->data + c->off[i], (size_t)(c->off[i + 1] - c->off[i]), c->out + 32 * i);
}
void oracle_hash_batch(int hasher, const uint8_t* data, const uint64_t* offsets, size_t n,
                       uint8_t* out32, int nthreads)
{
    hash_ctx c = {hasher, data, offsets, out32};
    oracle_parallel_for(n, nthreads, hash_range, &c);
}

typedef struct { const uint8_t *hash, *sig; uint8_t *pub, *ok; } rec_ctx;
static void rec_range(void* p, size_t lo, size_t hi)
{
    rec_ctx* c = (rec_ctx*)p;
    for (size_t i = lo; i < hi; ++i) {
        uint8_t pub[64];
        int r = oracle_secp256k1_recover(c->hash + 32 * i, c->sig + 65 * i, 65, pub);
        c->ok[i] = r == 0;
        if (c->pub) {
            if (r == 0) memcpy(c->pub + 64 * i, pub, 64);
            else memset(c->pub + 64 * i, 0, 64);
        }
    }
}
void oracle_secp256k1_recover_batch(const uint8_t* hash32, const uint8_t* sig65, size_t n,
                                    uint8_t* pub64, uint8_t* ok, int nthreads)
{
    uint8_t dummy[64];
    oracle_secp256k1_pubkey((const uint8_t*)"\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\1", dummy); /* init tables before threading */
    rec_ctx c = {hash32, sig65, pub64, ok};
    oracle_parallel_for(n, nthreads, rec_range, &c);
}

typedef struct { const uint8_t *hash, *sig; uint8_t* ok; } sm2_ctx;
static void sm2_range(void* p, size_t lo, size_t hi)
{
    sm2_ctx* c = (sm2_ctx*)p;
    for (size_t i = lo; i < hi; ++i)
        c->ok[i] = oracle_sm2_recover(c->hash + 32 * i, c->sig + 128 * i, 128, NULL) == 0;
}
void oracle_sm2_verify_batch(const uint8_t* hash32, const uint8_t* sig128, size_t n, uint8_t* ok,
                             int nthreads)
{
    uint8_t dummy[64];
    oracle_sm2_pubkey((const uint8_t*)"\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\1", dummy);
    sm2_ctx c = {hash32, sig128, ok};
    oracle_parallel_for(n, nthreads, sm2_range, &c);
}

typedef struct {
    int suite;
    const uint8_t *pre, *sig;
    const uint64_t *pre_off, *sig_off;
    uint8_t *txhash, *sender, *status;
} tx_ctx;
static void tx_range(void* p, size_t lo, size_t hi)
{
    tx_ctx* c = (tx_ctx*)p;
    int hasher = c->suite == ORACLE_SUITE_SM2 ? ORACLE_SM3 : ORACLE_KECCAK256;
    for (size_t i = lo; i < hi; ++i) {
        uint8_t* h = c->txhash + 32 * i;
        /* TarsHashable.h:16-41: tx hash = H(preimage) */
        oracle_hash(hasher, c->pre + c->pre_off[i], (size_t)(c->pre_off[i + 1] - c->pre_off[i]), h);
        const uint8_t* s = c->sig + c->sig_off[i];
        size_t slen = (size_t)(c->sig_off[i + 1] - c->sig_off[i]);
        uint8_t pub[64], ph[32];
        int r = c->suite == ORACLE_SUITE_SM2 ? oracle_sm2_recover(h, s, slen, pub)
                                             : oracle_secp256k1_recover(h, s, slen, pub);
        if (r == 0) { /* sender = right160(H(pub)) (Transaction.h:81, FixedBytes.h:666-671) */
            oracle_hash(hasher, pub, 64, ph);
            memcpy(c->sender + 20 * i, ph + 12, 20);
            c->status[i] = 0;
        } else {
            memset(c->sender + 20 * i, 0, 20);
            c->status[i] = 1; /* TransactionStatus::InvalidSignature (TxValidator.cpp:54-61) */
        }
    }
}
void oracle_tx_verify_batch(int suite, const uint8_t* pre, const uint64_t* pre_off,
                            const uint8_t* sig, const uint64_t* sig_off, size_t n,
                            uint8_t* txhash32, uint8_t* sender20, uint8_t* status, int nthreads)
{
    uint8_t dummy[64];
    oracle_sm2_pubkey((const uint8_t*)"\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\1", dummy);
    tx_ctx c = {suite, pre, sig, pre_off, sig_off, txhash32, sender20, status};
    oracle_parallel_for(n, nthreads, tx_range, &c);
}
