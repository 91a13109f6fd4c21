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
 *   hashes:    SM3 by EVP; Keccak-256 by the oracle's portable C (OpenSSL 1.1.1 has no pad-0x01
 *              Keccak EVP; the reference pokes its SHA3 context, OpenSSLHasher.h:51-80).
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
