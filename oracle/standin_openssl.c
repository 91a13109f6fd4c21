/*
 * standin_openssl.c -- the declared CPU stand-in for the reference's tx-admission path, timed as
 * bench.py's cpu_baseline.  TEST / BASELINE INFRASTRUCTURE ONLY: loaded by bench.py's
 * cpu_baseline leg and by tests/, never by the product (fisco-bcos_amd/).
 *
 * The reference verifies each transaction on a CPU thread pool: TransactionSync::importDownloadedTxs
 * runs tbb::parallel_for over the batch (bcos-txpool/bcos-txpool/sync/TransactionSync.cpp:516-548),
 * each iteration Transaction::verify (bcos-framework/bcos-framework/protocol/Transaction.h:68-82):
 * tx hash (TarsHashable.h:16-41), SignatureCrypto::recover, sender = right160(H(pub)).  The recover
 * itself is third-party code absent from /root/reference (wedpr-crypto's libsecp256k1 for
 * Secp256k1Crypto.cpp:79-93, TASSL sm2_do_verify for fast_sm2.cpp:139-227), so this restates the
 * same per-transaction work over OpenSSL 1.1.1's libcrypto EC (the /opt/conda build in this image):
 *   secp256k1: R from (r, v) by EC_POINT_set_compressed_coordinates, Q = (-e/r) G + (s/r) R by one
 *              EC_POINT_mul (OpenSSL's generic wNAF), pub = affine Q;
 *   SM2:       EVP_DigestVerify with SM3 and the user ID "1234567812345678" (fast_sm2.cpp:34,203) over
 *              the DER-encoded (r, s) and the 32-byte tx hash, against the embedded pubkey;
 *   hashes:    SM3 by EVP; Keccak-256 in the tx path by the oracle's portable C.
 * And the reference's Merkle CPU path (standin_merkle_root): Merkle<H, width>::generateMerkle
 * (Merkle.h:170-261) with its OpenSSL hashers (OpenSSLHasher.h:22-143, as merkleBench.cpp uses them) --
 * EVP_sm3, and EVP_sha3_256 with the KECCAK1600_CTX pad byte poked from 0x06 to 0x01 for Keccak-256,
 * exactly the reference's trick (OpenSSLHasher.h:51-80) -- levels computed in parallel like its
 * tbb::parallel_for, one hasher per range.
 * Contexts (EC_GROUP, BN_CTX) are per thread, as libsecp256k1's static context would be; the SM2 leg
 * builds its EVP objects per call, as fast_sm2_verify does (fast_sm2.cpp:139-227).
 * Verdicts equal the oracle's on well-formed signatures (tests/test_standin.py).
 */
#include "oracle.h"
#include "parallel.h"
#include <openssl/bn.h>
#include <openssl/crypto.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <stdlib.h>
#include <string.h>

const char* standin_version(void) { return OpenSSL_version(OPENSSL_VERSION); }

typedef struct {
    EC_GROUP* g;
    BN_CTX* ctx;
    BIGNUM *n, *p;
} k1_ctx;

static void k1_open(k1_ctx* c)
{
    c->g = EC_GROUP_new_by_curve_name(NID_secp256k1);
    c->ctx = BN_CTX_new();
    c->n = BN_new();
    c->p = BN_new();
    EC_GROUP_get_order(c->g, c->n, c->ctx);
    EC_GROUP_get_curve(c->g, c->p, NULL, NULL, c->ctx);
}

static void k1_close(k1_ctx* c)
{
    BN_free(c->n); BN_free(c->p); BN_CTX_free(c->ctx); EC_GROUP_free(c->g);
}

/* libsecp256k1 ecdsa_recover semantics (reject v > 3, r or s not in [1, n-1], v & 2 with
 * r + n >= p, x not on the curve, Q = infinity) over OpenSSL BN/EC */
static int k1_recover(k1_ctx* c, const uint8_t h[32], const uint8_t* sig, size_t siglen, uint8_t pub[64])
{
    if (siglen != 65 || sig[64] > 3) return -1;
    int ok = -1, v = sig[64];
    BN_CTX_start(c->ctx);
    BIGNUM *r = BN_CTX_get(c->ctx), *s = BN_CTX_get(c->ctx), *e = BN_CTX_get(c->ctx), *x = BN_CTX_get(c->ctx),
           *rinv = BN_CTX_get(c->ctx), *u1 = BN_CTX_get(c->ctx), *u2 = BN_CTX_get(c->ctx),
           *qx = BN_CTX_get(c->ctx), *qy = BN_CTX_get(c->ctx);
    EC_POINT *R = EC_POINT_new(c->g), *Q = EC_POINT_new(c->g);
    BN_bin2bn(sig, 32, r);
    BN_bin2bn(sig + 32, 32, s);
    BN_bin2bn(h, 32, e);
    if (BN_is_zero(r) || BN_is_zero(s) || BN_cmp(r, c->n) >= 0 || BN_cmp(s, c->n) >= 0) goto done;
    BN_copy(x, r);
    if (v & 2) BN_add(x, x, c->n);
    if (BN_cmp(x, c->p) >= 0) goto done;
    if (!EC_POINT_set_compressed_coordinates(c->g, R, x, v & 1, c->ctx)) goto done;
    BN_nnmod(e, e, c->n, c->ctx);
    if (!BN_mod_inverse(rinv, r, c->n, c->ctx)) goto done;
    BN_mod_mul(u1, e, rinv, c->n, c->ctx);
    BN_mod_sub(u1, c->n, u1, c->n, c->ctx);
    BN_mod_mul(u2, s, rinv, c->n, c->ctx);
    if (!EC_POINT_mul(c->g, Q, u1, R, u2, c->ctx) || EC_POINT_is_at_infinity(c->g, Q)) goto done;
    EC_POINT_get_affine_coordinates(c->g, Q, qx, qy, c->ctx);
    BN_bn2binpad(qx, pub, 32);
    BN_bn2binpad(qy, pub + 32, 32);
    ok = 0;
done:
    ERR_clear_error();
    EC_POINT_free(R);
    EC_POINT_free(Q);
    BN_CTX_end(c->ctx);
    return ok;
}

/* SM2Crypto::recover -> verify against the embedded key (SM2Crypto.cpp:66-92): sig = r||s||pub */
static int sm2_recover(const uint8_t h[32], const uint8_t* sig, size_t siglen, uint8_t pub[64])
{
    if (siglen != 128) return -1;
    int ok = 0;
    EC_KEY* k = EC_KEY_new_by_curve_name(NID_sm2);
    BIGNUM *x = BN_bin2bn(sig + 64, 32, NULL), *y = BN_bin2bn(sig + 96, 32, NULL);
    EVP_PKEY* pk = NULL;
    EVP_MD_CTX* m = NULL;
    EVP_PKEY_CTX* pc = NULL;
    ECDSA_SIG* sg = NULL;
    if (EC_KEY_set_public_key_affine_coordinates(k, x, y) != 1) goto done; /* pub on the curve, < p */
    pk = EVP_PKEY_new();
    EVP_PKEY_set1_EC_KEY(pk, k);
    EVP_PKEY_set_alias_type(pk, EVP_PKEY_SM2);
    m = EVP_MD_CTX_new();
    pc = EVP_PKEY_CTX_new(pk, NULL);
    EVP_PKEY_CTX_set1_id(pc, "1234567812345678", 16);
    EVP_MD_CTX_set_pkey_ctx(m, pc);
    sg = ECDSA_SIG_new();
    ECDSA_SIG_set0(sg, BN_bin2bn(sig, 32, NULL), BN_bin2bn(sig + 32, 32, NULL));
    uint8_t der[80], *q = der;
    int dl = i2d_ECDSA_SIG(sg, &q);
    if (EVP_DigestVerifyInit(m, NULL, EVP_sm3(), NULL, pk) == 1)
        ok = EVP_DigestVerify(m, der, (size_t)dl, h, 32) == 1;
done:
    ERR_clear_error();
    ECDSA_SIG_free(sg);
    EVP_MD_CTX_free(m);
    EVP_PKEY_CTX_free(pc);
    EVP_PKEY_free(pk);
    BN_free(x);
    BN_free(y);
    EC_KEY_free(k);
    if (!ok) return -1;
    memcpy(pub, sig + 64, 64);
    return 0;
}

static void sm3_evp(const uint8_t* in, size_t len, uint8_t out[32])
{
    unsigned int ol = 32;
    EVP_Digest(in, len, out, &ol, EVP_sm3(), NULL);
}

typedef struct {
    int suite;
    const uint8_t *pre, *sig;
    const uint64_t *pre_off, *sig_off;
    uint8_t *txhash, *sender, *status;
} tx_job;

static void tx_range(void* p, size_t lo, size_t hi)
{
    tx_job* j = (tx_job*)p;
    k1_ctx c = {0};
    if (j->suite == ORACLE_SUITE_SECP256K1) k1_open(&c);
    for (size_t i = lo; i < hi; ++i) {
        const uint8_t* m = j->pre + j->pre_off[i];
        const size_t ml = (size_t)(j->pre_off[i + 1] - j->pre_off[i]);
        const uint8_t* s = j->sig + j->sig_off[i];
        const size_t sl = (size_t)(j->sig_off[i + 1] - j->sig_off[i]);
        uint8_t* th = j->txhash + 32 * i;
        uint8_t pub[64], d[32];
        int rc;
        if (j->suite == ORACLE_SUITE_SECP256K1) {
            oracle_keccak256(m, ml, th);
            rc = k1_recover(&c, th, s, sl, pub);
            if (!rc) oracle_keccak256(pub, 64, d);
        } else {
            sm3_evp(m, ml, th);
            rc = sm2_recover(th, s, sl, pub);
            if (!rc) sm3_evp(pub, 64, d);
        }
        if (rc) memset(d, 0, 32);
        memcpy(j->sender + 20 * i, d + 12, 20);
        j->status[i] = rc ? 1 : 0;
    }
    if (j->suite == ORACLE_SUITE_SECP256K1) k1_close(&c);
}

/* Transaction::verify over a batch on nthreads threads (contiguous shards, TransactionSync.cpp:516) */
void standin_tx_verify_batch(int suite, const uint8_t* pre, const uint64_t* pre_off, const uint8_t* sig,
                             const uint64_t* sig_off, size_t n, uint8_t* txhash32, uint8_t* sender20,
                             uint8_t* status, int nthreads)
{
    tx_job j = {suite, pre, sig, pre_off, sig_off, txhash32, sender20, status};
    oracle_parallel_for(n, nthreads, tx_range, &j);
}

/* ------------------------------------------------------------------ verify with a known key */
/* secp256k1Verify -> wedpr_secp256k1_verify (Secp256k1Crypto.cpp:51-63), libsecp256k1 ecdsa_verify
 * semantics over OpenSSL: key on the curve, r, s in [1, n-1], low-S (s <= n/2), ECDSA_do_verify */
static int k1_verify(k1_ctx* c, const uint8_t pub[64], const uint8_t h[32], const uint8_t sig[64])
{
    int ok = 0;
    EC_KEY* k = EC_KEY_new();
    BIGNUM *x = BN_bin2bn(pub, 32, NULL), *y = BN_bin2bn(pub + 32, 32, NULL);
    BIGNUM *r = BN_bin2bn(sig, 32, NULL), *s = BN_bin2bn(sig + 32, 32, NULL), *half = BN_new();
    ECDSA_SIG* sg = NULL;
    BN_rshift1(half, c->n);
    if (BN_is_zero(r) || BN_is_zero(s) || BN_cmp(r, c->n) >= 0 || BN_cmp(s, half) > 0) goto done;
    EC_KEY_set_group(k, c->g);
    if (EC_KEY_set_public_key_affine_coordinates(k, x, y) != 1) goto done;
    sg = ECDSA_SIG_new();
    ECDSA_SIG_set0(sg, r, s);
    r = s = NULL;
    ok = ECDSA_do_verify(h, 32, sg, k) == 1;
done:
    ERR_clear_error();
    ECDSA_SIG_free(sg);
    BN_free(r);
    BN_free(s);
    BN_free(half);
    BN_free(x);
    BN_free(y);
    EC_KEY_free(k);
    return ok;
}

typedef struct {
    int suite;
    const uint8_t *pub, *hash, *sig;
    size_t stride;
    uint8_t* ok;
} verify_job;

static void verify_range(void* p, size_t lo, size_t hi)
{
    verify_job* j = (verify_job*)p;
    k1_ctx c = {0};
    if (j->suite == ORACLE_SUITE_SECP256K1) k1_open(&c);
    for (size_t i = lo; i < hi; ++i) {
        const uint8_t* s = j->sig + j->stride * i;
        if (j->suite == ORACLE_SUITE_SECP256K1) {
            j->ok[i] = (uint8_t)k1_verify(&c, j->pub + 64 * i, j->hash + 32 * i, s);
        } else { /* SM2Crypto::verify (SM2Crypto.cpp:66-79): r || s = sig[0..64), the given key */
            uint8_t rsp[128], out[64];
            memcpy(rsp, s, 64);
            memcpy(rsp + 64, j->pub + 64 * i, 64);
            j->ok[i] = sm2_recover(j->hash + 32 * i, rsp, 128, out) == 0;
        }
    }
    if (j->suite == ORACLE_SUITE_SECP256K1) k1_close(&c);
}

/* SignatureCrypto::verify(pub, hash, sig) over a batch on nthreads threads (the sealer-signature checks,
 * BlockValidator.cpp:141-182) */
void standin_verify_batch(int suite, const uint8_t* pub64, const uint8_t* hash32, const uint8_t* sig, size_t stride,
                          size_t n, uint8_t* ok, int nthreads)
{
    verify_job j = {suite, pub64, hash32, sig, stride, ok};
    oracle_parallel_for(n, nthreads, verify_range, &j);
}

/* ------------------------------------------------------------------ the reference's Merkle CPU path */
/* OpenSSL 1.1.1's KECCAK1600_CTX and EVP_MD_CTX head (the layout OpenSSLHasher.h:51-75 relies on) */
typedef struct {
    uint64_t A[5][5];
    size_t block_size;
    size_t md_size;
    size_t num;
    unsigned char buf[1600 / 8 - 32];
    unsigned char pad;
} standin_keccak1600_ctx;
typedef struct {
    const EVP_MD* digest;
    void* engine;
    unsigned long flags;
    standin_keccak1600_ctx* md_data;
} standin_evp_md_ctx_head;

/* OpenSSLHasher<H>::init: EVP_DigestInit, and for Keccak-256 the pad poke; 0 on a layout mismatch */
static int ossl_hasher_init(EVP_MD_CTX* m, int hasher)
{
    if (hasher == ORACLE_SM3) return EVP_DigestInit(m, EVP_sm3()) == 1;
    if (EVP_DigestInit(m, EVP_sha3_256()) != 1) return 0;
    standin_evp_md_ctx_head* h = (standin_evp_md_ctx_head*)m;
    if (!h->md_data || h->md_data->pad != 0x06) return 0;
    h->md_data->pad = 0x01;
    return 1;
}

int standin_hash(int hasher, const uint8_t* in, size_t len, uint8_t out[32])
{
    EVP_MD_CTX* m = EVP_MD_CTX_new();
    int ok = m && ossl_hasher_init(m, hasher) && EVP_DigestUpdate(m, in, len) == 1 &&
             EVP_DigestFinal(m, out, NULL) == 1;
    EVP_MD_CTX_free(m);
    return ok ? 0 : -1;
}

typedef struct {
    int hasher, width, fail;
    const uint8_t* in;
    size_t nin;
    uint8_t* out;
} level_job;

/* calculateLevelHashes (Merkle.h:243-261): one hasher per range, node i = H(in[i*w] .. in[i*w+w-1]) */
static void level_range(void* p, size_t lo, size_t hi)
{
    level_job* j = (level_job*)p;
    EVP_MD_CTX* m = EVP_MD_CTX_new();
    for (size_t i = lo; i < hi; ++i) {
        const size_t a = i * (size_t)j->width, b = a + (size_t)j->width < j->nin ? a + (size_t)j->width : j->nin;
        if (!m || !ossl_hasher_init(m, j->hasher) || EVP_DigestUpdate(m, j->in + 32 * a, 32 * (b - a)) != 1 ||
            EVP_DigestFinal(m, j->out + 32 * i, NULL) != 1)
            j->fail = 1;
    }
    EVP_MD_CTX_free(m);
}

/* Merkle<H, width>::generateMerkle's root over n 32-byte leaves on nthreads threads (levels in
 * sequence, each level's nodes in parallel).  Returns 0, or -1 (n == 0 / OpenSSL layout mismatch). */
int standin_merkle_root(int hasher, int width, const uint8_t* leaves, size_t n, uint8_t root[32], int nthreads)
{
    if (n == 0 || width < 2) return -1;
    if (n == 1) {
        memcpy(root, leaves, 32);
        return 0;
    }
    size_t cap = (n + (size_t)width - 1) / (size_t)width;
    uint8_t* a = (uint8_t*)malloc(32 * cap);
    uint8_t* b = (uint8_t*)malloc(32 * cap);
    int rc = a && b ? 0 : -1;
    const uint8_t* in = leaves;
    size_t nin = n;
    uint8_t* out = a;
    while (!rc && nin > 1) {
        const size_t nout = (nin + (size_t)width - 1) / (size_t)width;
        level_job j = {hasher, width, 0, in, nin, out};
        oracle_parallel_for(nout, nthreads, level_range, &j);
        if (j.fail) rc = -1;
        in = out;
        nin = nout;
        out = out == a ? b : a;
    }
    if (!rc) memcpy(root, in, 32);
    free(a);
    free(b);
    return rc;
}
