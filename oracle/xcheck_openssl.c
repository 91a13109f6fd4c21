/*
 * xcheck_openssl.c -- cross-checks the oracle's ECC restatement against an independent
 * implementation (OpenSSL 1.1.1 EC from /opt/conda, the SURVEY §8c stand-in for wedpr/TASSL), and
 * writes OpenSSL-computed golden vectors to tests/golden/ecc_openssl.json.
 * TEST INFRASTRUCTURE ONLY; built in the build container by `make -C oracle xcheck`
 * (output in oracle/_ref/), never shipped or run on the GPU box.
 *
 * usage: xcheck_openssl <n_random_checks> <fixture_json_path>
 */
#include "oracle.h"
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/rand.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void hexs(FILE* f, const uint8_t* b, size_t n)
{
    for (size_t i = 0; i < n; ++i) fprintf(f, "%02x", b[i]);
}

/* secp256k1 recovery with OpenSSL BN/EC: x = r (+n if v&2), R from compressed x, Q = r^-1(sR - eG) */
static int ossl_recover(const uint8_t h[32], const uint8_t sig[65], uint8_t pub[64])
{
    int ok = -1, v = sig[64];
    if (v > 3) return -1;
    BN_CTX* ctx = BN_CTX_new();
    EC_GROUP* g = EC_GROUP_new_by_curve_name(NID_secp256k1);
    BIGNUM *r = BN_bin2bn(sig, 32, NULL), *s = BN_bin2bn(sig + 32, 32, NULL),
           *e = BN_bin2bn(h, 32, NULL), *x = BN_new(), *n = BN_new(), *p = BN_new(),
           *rinv = BN_new(), *u1 = BN_new(), *u2 = BN_new(), *qx = BN_new(), *qy = BN_new();
    EC_POINT *R = EC_POINT_new(g), *Q = EC_POINT_new(g);
    EC_GROUP_get_order(g, n, ctx);
    EC_GROUP_get_curve(g, p, NULL, NULL, ctx);
    if (BN_is_zero(r) || BN_is_zero(s) || BN_cmp(r, n) >= 0 || BN_cmp(s, n) >= 0) goto done;
    BN_copy(x, r);
    if (v & 2) BN_add(x, x, n);
    if (BN_cmp(x, p) >= 0) goto done;
    if (!EC_POINT_set_compressed_coordinates(g, R, x, v & 1, ctx)) goto done;
    BN_mod(e, e, n, ctx);
    BN_mod_inverse(rinv, r, n, ctx);
    BN_mod_mul(u1, e, rinv, n, ctx);
    BN_sub(u1, n, u1);
    BN_mod(u1, u1, n, ctx);
    BN_mod_mul(u2, s, rinv, n, ctx);
    if (!EC_POINT_mul(g, Q, u1, R, u2, ctx)) goto done;
    if (EC_POINT_is_at_infinity(g, Q)) goto done;
    EC_POINT_get_affine_coordinates(g, Q, qx, qy, ctx);
    BN_bn2binpad(qx, pub, 32);
    BN_bn2binpad(qy, pub + 32, 32);
    ok = 0;
done:
    ERR_clear_error();
    BN_free(r); BN_free(s); BN_free(e); BN_free(x); BN_free(n); BN_free(p); BN_free(rinv);
    BN_free(u1); BN_free(u2); BN_free(qx); BN_free(qy);
    EC_POINT_free(R); EC_POINT_free(Q); EC_GROUP_free(g); BN_CTX_free(ctx);
    return ok;
}

static EVP_PKEY* sm2_key(const uint8_t sk[32], uint8_t pub[64])
{
    EC_KEY* k = EC_KEY_new_by_curve_name(NID_sm2);
    BIGNUM* d = BN_bin2bn(sk, 32, NULL);
    const EC_GROUP* g = EC_KEY_get0_group(k);
    EC_POINT* P = EC_POINT_new(g);
    EC_POINT_mul(g, P, d, NULL, NULL, NULL);
    EC_KEY_set_private_key(k, d);
    EC_KEY_set_public_key(k, P);
    BIGNUM *x = BN_new(), *y = BN_new();
    EC_POINT_get_affine_coordinates(g, P, x, y, NULL);
    BN_bn2binpad(x, pub, 32);
    BN_bn2binpad(y, pub + 32, 32);
    EVP_PKEY* pk = EVP_PKEY_new();
    EVP_PKEY_set1_EC_KEY(pk, k);
    EVP_PKEY_set_alias_type(pk, EVP_PKEY_SM2);
    BN_free(x); BN_free(y); BN_free(d); EC_POINT_free(P); EC_KEY_free(k);
    return pk;
}

/* OpenSSL SM2 sign/verify over the 32-byte tx hash with ID "1234567812345678" */
static int sm2_do(EVP_PKEY* pk, int sign, const uint8_t h[32], uint8_t rs[64])
{
    EVP_MD_CTX* m = EVP_MD_CTX_new();
    EVP_PKEY_CTX* pc = EVP_PKEY_CTX_new(pk, NULL);
    EVP_PKEY_CTX_set1_id(pc, "1234567812345678", 16);
    EVP_MD_CTX_set_pkey_ctx(m, pc);
    int ok = 0;
    if (sign) {
        uint8_t der[128];
        size_t dl = sizeof(der);
        EVP_DigestSignInit(m, NULL, EVP_sm3(), NULL, pk);
        ok = EVP_DigestSign(m, der, &dl, h, 32) == 1;
        const uint8_t* q = der;
        ECDSA_SIG* sg = d2i_ECDSA_SIG(NULL, &q, (long)dl);
        BN_bn2binpad(ECDSA_SIG_get0_r(sg), rs, 32);
        BN_bn2binpad(ECDSA_SIG_get0_s(sg), rs + 32, 32);
        ECDSA_SIG_free(sg);
    } else {
        ECDSA_SIG* sg = ECDSA_SIG_new();
        ECDSA_SIG_set0(sg, BN_bin2bn(rs, 32, NULL), BN_bin2bn(rs + 32, 32, NULL));
        uint8_t der[128], *q = der;
        int dl = i2d_ECDSA_SIG(sg, &q);
        EVP_DigestVerifyInit(m, NULL, EVP_sm3(), NULL, pk);
        ok = EVP_DigestVerify(m, der, (size_t)dl, h, 32) == 1;
        ECDSA_SIG_free(sg);
    }
    ERR_clear_error();
    EVP_MD_CTX_free(m);
    EVP_PKEY_CTX_free(pc);
    return ok;
}

int main(int argc, char** argv)
{
    int n = argc > 1 ? atoi(argv[1]) : 200;
    FILE* fx = argc > 2 ? fopen(argv[2], "w") : NULL;
    int bad = 0;
    if (fx) fprintf(fx, "{\n \"generator\": \"oracle/xcheck_openssl.c (OpenSSL %s)\",\n \"secp256k1_recover\": [\n", OPENSSL_VERSION_TEXT);
    /* secp256k1: oracle-signed (random key, hash, nonce) -> OpenSSL + oracle recover; plus
     * random garbage (r, s, v) where both must agree on failure/success and the key. */
    for (int i = 0; i < n; ++i) {
        uint8_t sk[32], h[32], k[32], sig[65], p1[64], p2[64], pub[64];
        RAND_bytes(sk, 32); RAND_bytes(h, 32); RAND_bytes(k, 32);
        if (i % 8 == 7) memset(h, 0, 32); /* e = 0 -> u1 = 0 */
        if (oracle_secp256k1_pubkey(sk, pub) || oracle_secp256k1_sign(sk, h, k, sig)) continue;
        int kind = i % 4; /* 0 valid, 1 random r/s/v, 2 flipped s bit, 3 v+2 */
        if (kind == 1) { RAND_bytes(sig, 64); sig[64] = (uint8_t)(i % 5); }
        if (kind == 2) sig[32 + (i % 32)] ^= (uint8_t)(1u << (i % 8));
        if (kind == 3) sig[64] ^= 2;
        int a = oracle_secp256k1_recover(h, sig, 65, p1), b = ossl_recover(h, sig, p2);
        if (kind == 0 && (a || memcmp(p1, pub, 64))) { ++bad; printf("secp valid mismatch %d\n", i); }
        if (a != b || (a == 0 && memcmp(p1, p2, 64))) { ++bad; printf("secp mismatch %d kind %d (%d,%d)\n", i, kind, a, b); }
        if (kind == 0 && oracle_secp256k1_verify(pub, h, sig, 65)) { ++bad; printf("secp verify %d\n", i); }
        if (fx && i < 96) {
            fprintf(fx, "  {\"hash\": \""); hexs(fx, h, 32);
            fprintf(fx, "\", \"sig\": \""); hexs(fx, sig, 65);
            fprintf(fx, "\", \"ok\": %s, \"pub\": \"", b == 0 ? "true" : "false");
            if (b == 0) hexs(fx, p2, 64);
            fprintf(fx, "\"}%s\n", i + 1 < 96 && i + 1 < n ? "," : "");
        }
    }
    if (fx) fprintf(fx, " ],\n \"sm2_verify\": [\n");
    for (int i = 0; i < n; ++i) {
        uint8_t sk[32], h[32], k[32], sig[128], pub[64], rs[64];
        RAND_bytes(sk, 32); RAND_bytes(h, 32); RAND_bytes(k, 32);
        sk[0] &= 0x7f;
        EVP_PKEY* pk = sm2_key(sk, pub);
        uint8_t opub[64];
        if (oracle_sm2_pubkey(sk, opub) || memcmp(opub, pub, 64)) { ++bad; printf("sm2 pub %d\n", i); }
        int kind = i % 4; /* 0 OpenSSL-signed, 1 oracle-signed, 2 flipped bit, 3 wrong hash */
        if (kind == 1) { if (oracle_sm2_sign(sk, h, k, sig)) { EVP_PKEY_free(pk); continue; } memcpy(rs, sig, 64); }
        else sm2_do(pk, 1, h, rs);
        memcpy(sig, rs, 64); memcpy(sig + 64, pub, 64);
        if (kind == 2) sig[i % 128] ^= (uint8_t)(1u << (i % 8));
        if (kind == 3) h[i % 32] ^= 1;
        int a = oracle_sm2_recover(h, sig, 128, NULL) == 0;
        int b;
        if (kind == 2 && (i % 128) >= 64) { /* corrupted pubkey: OpenSSL key parse decides */
            EC_KEY* ek = EC_KEY_new_by_curve_name(NID_sm2);
            EC_POINT* P = EC_POINT_new(EC_KEY_get0_group(ek));
            BIGNUM *x = BN_bin2bn(sig + 64, 32, NULL), *y = BN_bin2bn(sig + 96, 32, NULL);
            int on = EC_POINT_set_affine_coordinates(EC_KEY_get0_group(ek), P, x, y, NULL);
            b = 0;
            if (on) {
                EC_KEY_set_public_key(ek, P);
                EVP_PKEY* pk2 = EVP_PKEY_new();
                EVP_PKEY_set1_EC_KEY(pk2, ek);
                EVP_PKEY_set_alias_type(pk2, EVP_PKEY_SM2);
                b = sm2_do(pk2, 0, h, sig);
                EVP_PKEY_free(pk2);
            }
            ERR_clear_error();
            BN_free(x); BN_free(y); EC_POINT_free(P); EC_KEY_free(ek);
        } else b = sm2_do(pk, 0, h, sig);
        if (a != b) { ++bad; printf("sm2 mismatch %d kind %d (%d,%d)\n", i, kind, a, b); }
        if (kind < 2 && !a) { ++bad; printf("sm2 valid rejected %d\n", i); }
        if (fx && i < 96) {
            fprintf(fx, "  {\"hash\": \""); hexs(fx, h, 32);
            fprintf(fx, "\", \"sig\": \""); hexs(fx, sig, 128);
            fprintf(fx, "\", \"ok\": %s}%s\n", b ? "true" : "false", i + 1 < 96 && i + 1 < n ? "," : "");
        }
        EVP_PKEY_free(pk);
    }
    if (fx) { fprintf(fx, " ]\n}\n"); fclose(fx); }
    printf("xcheck: %d random cases per curve, %d mismatches\n", n, bad);
    return bad ? 1 : 0;
}
