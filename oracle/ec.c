/*
 * ec.c -- oracle restatement of the ECC the reference delegates to third-party code.
 * TEST INFRASTRUCTURE ONLY.
 *
 * The reference calls (bcos-crypto/bcos-crypto/signature/):
 *   secp256k1: wedpr_secp256k1_recover_public_key / _verify / _sign   (Secp256k1Crypto.cpp:33-93)
 *              -> wedpr-crypto (Rust, FISCO vcpkg registry, vcpkg.json:48) -> libsecp256k1.
 *   SM2:       fast_sm2_verify -> TASSL sm2_do_verify(EVP_sm3, id "1234567812345678")
 *              (fastsm2/fast_sm2.cpp:34,139-227), wedpr_sm2_verify (sm2/SM2Crypto.h:39).
 * Neither third-party library is present in /root/reference, so this file restates their
 * published algorithms (libsecp256k1 secp256k1_ecdsa_recover / sig_verify / sig_sign; GB/T 32918.2
 * as implemented by OpenSSL/TASSL sm2_sig_verify) with generic 4x64-bit Montgomery arithmetic --
 * deliberately a DIFFERENT arithmetic than the HIP kernels (8x32-bit limbs, pseudo-Mersenne
 * reduction) so that a shared bug is unlikely.  Pinned by the reference's KATs
 * (SignatureTest.cpp:53-63,238-251; EVMPrecompiledTest.cpp:58-72) and cross-checked against
 * OpenSSL 1.1.1 EC by oracle/xcheck_openssl.c.
 */
#include "oracle.h"
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256; /* little-endian 64-bit limbs */

static void u256_from_be(u256* r, const uint8_t b[32])
{
    for (int i = 0; i < 4; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
        r->v[i] = w;
    }
}
static void u256_to_be(uint8_t b[32], const u256* a)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256* a, const u256* b)
{
    for (int i = 3; i >= 0; --i) {
        if (a->v[i] < b->v[i]) return -1;
        if (a->v[i] > b->v[i]) return 1;
    }
    return 0;
}
static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static uint64_t u256_add(u256* r, const u256* a, const u256* b)
{
    u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b)
{
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->v[i] - b->v[i] - borrow;
        r->v[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 127);
    }
    return borrow;
}
static int u256_bit(const u256* a, int i) { return (int)((a->v[i >> 6] >> (i & 63)) & 1); }

/* ---------------- Montgomery arithmetic modulo an odd 256-bit m, R = 2^256 ---------------- */
typedef struct { u256 m, r2, one; uint64_t minv; } mont;

static void mod_add(const mont* c, u256* r, const u256* a, const u256* b)
{
    uint64_t carry = u256_add(r, a, b);
    if (carry || u256_cmp(r, &c->m) >= 0) u256_sub(r, r, &c->m);
}
static void mod_sub(const mont* c, u256* r, const u256* a, const u256* b)
{
    if (u256_sub(r, a, b)) u256_add(r, r, &c->m);
}
static void mod_neg(const mont* c, u256* r, const u256* a)
{
    u256 z = {{0, 0, 0, 0}};
    mod_sub(c, r, &z, a);
}
static void mont_mul(const mont* c, u256* r, const u256* a, const u256* b)
{
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) { /* CIOS */
        u128 C = 0;
        for (int j = 0; j < 4; ++j) {
            C += (u128)a->v[j] * b->v[i] + t[j];
            t[j] = (uint64_t)C; C >>= 64;
        }
        C += t[4]; t[4] = (uint64_t)C; t[5] = (uint64_t)(C >> 64);
        uint64_t m = t[0] * c->minv;
        C = (u128)m * c->m.v[0] + t[0];
        C >>= 64;
        for (int j = 1; j < 4; ++j) {
            C += (u128)m * c->m.v[j] + t[j];
            t[j - 1] = (uint64_t)C; C >>= 64;
        }
        C += t[4]; t[3] = (uint64_t)C; C >>= 64;
        t[4] = t[5] + (uint64_t)C;
    }
    u256 res = {{t[0], t[1], t[2], t[3]}};
    if (t[4] || u256_cmp(&res, &c->m) >= 0) u256_sub(&res, &res, &c->m);
    *r = res;
}
static void mont_init(mont* c, const u256* m)
{
    c->m = *m;
    uint64_t inv = 1; /* Newton: inv = m0^-1 mod 2^64 */
    for (int i = 0; i < 7; ++i) inv *= 2 - m->v[0] * inv;
    c->minv = (uint64_t)0 - inv;
    u256 x = {{1, 0, 0, 0}};
    for (int i = 0; i < 512; ++i) {
        if (i == 256) c->one = x;
        mod_add(c, &x, &x, &x);
    }
    c->r2 = x;
}
static void to_mont(const mont* c, u256* r, const u256* a) { mont_mul(c, r, a, &c->r2); }
static void from_mont(const mont* c, u256* r, const u256* a)
{
    u256 one = {{1, 0, 0, 0}};
    mont_mul(c, r, a, &one);
}
static void mont_pow(const mont* c, u256* r, const u256* a, const u256* e)
{
    u256 acc = c->one;
    for (int i = 255; i >= 0; --i) {
        mont_mul(c, &acc, &acc, &acc);
        if (u256_bit(e, i)) mont_mul(c, &acc, &acc, a);
    }
    *r = acc;
}
static void mont_inv(const mont* c, u256* r, const u256* a)
{
    u256 e, two = {{2, 0, 0, 0}};
    u256_sub(&e, &c->m, &two); /* Fermat: a^(m-2) */
    mont_pow(c, r, a, &e);
}

/* ---------------- short Weierstrass curves y^2 = x^3 + a x + b ---------------- */
typedef struct { mont p, n; u256 a, b, gx, gy; /* Montgomery form mod p */ u256 n_plain; } curve;
typedef struct { u256 X, Y, Z; } jpt; /* Jacobian, Montgomery form; Z == 0 => infinity */

static curve g_secp, g_sm2;
static int g_init = 0;

static void hex_to_u256(u256* r, const char* hex)
{
    uint8_t b[32];
    for (int i = 0; i < 32; ++i) {
        int hi = hex[2 * i], lo = hex[2 * i + 1];
        hi = hi <= '9' ? hi - '0' : (hi | 32) - 'a' + 10;
        lo = lo <= '9' ? lo - '0' : (lo | 32) - 'a' + 10;
        b[i] = (uint8_t)(hi * 16 + lo);
    }
    u256_from_be(r, b);
}
static void curve_setup(curve* C, const char* p, const char* n, const char* a, const char* b,
                        const char* gx, const char* gy)
{
    u256 t;
    hex_to_u256(&t, p); mont_init(&C->p, &t);
    hex_to_u256(&t, n); mont_init(&C->n, &t); C->n_plain = t;
    hex_to_u256(&t, a); to_mont(&C->p, &C->a, &t);
    hex_to_u256(&t, b); to_mont(&C->p, &C->b, &t);
    hex_to_u256(&t, gx); to_mont(&C->p, &C->gx, &t);
    hex_to_u256(&t, gy); to_mont(&C->p, &C->gy, &t);
}
static void ec_init(void)
{
    if (g_init) return;
    /* secp256k1 (SEC 2) -- curve of Secp256k1Crypto */
    curve_setup(&g_secp, "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F",
                "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141",
                "0000000000000000000000000000000000000000000000000000000000000000",
                "0000000000000000000000000000000000000000000000000000000000000007",
                "79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798",
                "483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8");
    /* SM2 recommended curve (GB/T 32918.5), NID_sm2 of fast_sm2.cpp:40 */
    curve_setup(&g_sm2, "FFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF00000000FFFFFFFFFFFFFFFF",
                "FFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123",
                "FFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF00000000FFFFFFFFFFFFFFFC",
                "28E9FA9E9D9F5E344D5A9E4BCF6509A7F39789F515AB8F92DDBCBD414D940E93",
                "32C4AE2C1F1981195F9904466A39C9948FE30BBFF2660BE1715A4589334C74C7",
                "BC3736A2F4F6779C59BDCEE36B692153D0A9877CC62A474002DF32E52139F0A0");
    g_init = 1;
}

static int pt_is_inf(const jpt* P) { return u256_is_zero(&P->Z); }
static void pt_set_inf(jpt* P) { memset(P, 0, sizeof(*P)); }

/* dbl-2007-bl with general a (M = 3X^2 + a Z^4) */
static void pt_dbl(const curve* C, jpt* R, const jpt* P)
{
    const mont* f = &C->p;
    if (pt_is_inf(P) || u256_is_zero(&P->Y)) { pt_set_inf(R); return; }
    u256 XX, YY, YYYY, ZZ, S, M, T, X3, Y3, Z3;
    mont_mul(f, &XX, &P->X, &P->X);
    mont_mul(f, &YY, &P->Y, &P->Y);
    mont_mul(f, &YYYY, &YY, &YY);
    mont_mul(f, &ZZ, &P->Z, &P->Z);
    mod_add(f, &T, &P->X, &YY);
    mont_mul(f, &S, &T, &T);
    mod_sub(f, &S, &S, &XX);
    mod_sub(f, &S, &S, &YYYY);
    mod_add(f, &S, &S, &S);
    mod_add(f, &M, &XX, &XX);
    mod_add(f, &M, &M, &XX);
    mont_mul(f, &T, &ZZ, &ZZ);
    mont_mul(f, &T, &T, &C->a);
    mod_add(f, &M, &M, &T);
    mont_mul(f, &X3, &M, &M);
    mod_sub(f, &X3, &X3, &S);
    mod_sub(f, &X3, &X3, &S);
    mod_sub(f, &T, &S, &X3);
    mont_mul(f, &Y3, &M, &T);
    mod_add(f, &T, &YYYY, &YYYY);
    mod_add(f, &T, &T, &T);
    mod_add(f, &T, &T, &T);
    mod_sub(f, &Y3, &Y3, &T);
    mod_add(f, &T, &P->Y, &P->Z);
    mont_mul(f, &Z3, &T, &T);
    mod_sub(f, &Z3, &Z3, &YY);
    mod_sub(f, &Z3, &Z3, &ZZ);
    R->X = X3; R->Y = Y3; R->Z = Z3;
}

/* complete-case Jacobian addition (handles infinity, P == Q, P == -Q) */
static void pt_add(const curve* C, jpt* R, const jpt* P, const jpt* Q)
{
    const mont* f = &C->p;
    if (pt_is_inf(P)) { *R = *Q; return; }
    if (pt_is_inf(Q)) { *R = *P; return; }
    u256 Z1Z1, Z2Z2, U1, U2, S1, S2, H, r, HH, HHH, V, T, X3, Y3, Z3;
    mont_mul(f, &Z1Z1, &P->Z, &P->Z);
    mont_mul(f, &Z2Z2, &Q->Z, &Q->Z);
    mont_mul(f, &U1, &P->X, &Z2Z2);
    mont_mul(f, &U2, &Q->X, &Z1Z1);
    mont_mul(f, &S1, &P->Y, &Q->Z);
    mont_mul(f, &S1, &S1, &Z2Z2);
    mont_mul(f, &S2, &Q->Y, &P->Z);
    mont_mul(f, &S2, &S2, &Z1Z1);
    mod_sub(f, &H, &U2, &U1);
    mod_sub(f, &r, &S2, &S1);
    if (u256_is_zero(&H)) {
        if (u256_is_zero(&r)) { pt_dbl(C, R, P); return; }
        pt_set_inf(R);
        return;
    }
    mont_mul(f, &HH, &H, &H);
    mont_mul(f, &HHH, &H, &HH);
    mont_mul(f, &V, &U1, &HH);
    mont_mul(f, &X3, &r, &r);
    mod_sub(f, &X3, &X3, &HHH);
    mod_sub(f, &X3, &X3, &V);
    mod_sub(f, &X3, &X3, &V);
    mod_sub(f, &T, &V, &X3);
    mont_mul(f, &Y3, &r, &T);
    mont_mul(f, &T, &S1, &HHH);
    mod_sub(f, &Y3, &Y3, &T);
    mont_mul(f, &Z3, &P->Z, &Q->Z);
    mont_mul(f, &Z3, &Z3, &H);
    R->X = X3; R->Y = Y3; R->Z = Z3;
}

/* k1*P1 + k2*P2, joint 4-bit fixed windows (Straus) */
static void pt_mul2(const curve* C, jpt* R, const u256* k1, const jpt* P1, const u256* k2,
                    const jpt* P2)
{
    jpt T1[16], T2[16], acc;
    pt_set_inf(&T1[0]); pt_set_inf(&T2[0]);
    T1[1] = *P1; T2[1] = *P2;
    for (int i = 2; i < 16; ++i) {
        pt_add(C, &T1[i], &T1[i - 1], P1);
        pt_add(C, &T2[i], &T2[i - 1], P2);
    }
    pt_set_inf(&acc);
    for (int w = 63; w >= 0; --w) {
        for (int d = 0; d < 4; ++d) pt_dbl(C, &acc, &acc);
        int n1 = (int)((k1->v[w / 16] >> (4 * (w % 16))) & 15);
        int n2 = (int)((k2->v[w / 16] >> (4 * (w % 16))) & 15);
        if (n1) pt_add(C, &acc, &acc, &T1[n1]);
        if (n2) pt_add(C, &acc, &acc, &T2[n2]);
    }
    *R = acc;
}

/* affine (plain, not Montgomery) coordinates; -1 if infinity */
static int pt_affine(const curve* C, u256* x, u256* y, const jpt* P)
{
    const mont* f = &C->p;
    if (pt_is_inf(P)) return -1;
    u256 zi, zi2, zi3, t;
    mont_inv(f, &zi, &P->Z);
    mont_mul(f, &zi2, &zi, &zi);
    mont_mul(f, &zi3, &zi2, &zi);
    mont_mul(f, &t, &P->X, &zi2);
    from_mont(f, x, &t);
    mont_mul(f, &t, &P->Y, &zi3);
    from_mont(f, y, &t);
    return 0;
}

/* plain affine coordinates -> Jacobian point; -1 if a coordinate >= p or the point is off-curve */
static int pt_from_affine(const curve* C, jpt* P, const u256* x, const u256* y)
{
    const mont* f = &C->p;
    if (u256_cmp(x, &f->m) >= 0 || u256_cmp(y, &f->m) >= 0) return -1;
    u256 xm, ym, lhs, rhs, t;
    to_mont(f, &xm, x);
    to_mont(f, &ym, y);
    mont_mul(f, &lhs, &ym, &ym);
    mont_mul(f, &rhs, &xm, &xm);
    mod_add(f, &rhs, &rhs, &C->a);
    mont_mul(f, &rhs, &rhs, &xm);
    mod_add(f, &rhs, &rhs, &C->b);
    (void)t;
    if (u256_cmp(&lhs, &rhs) != 0) return -1;
    P->X = xm; P->Y = ym; P->Z = f->one;
    return 0;
}

static void gen_point(const curve* C, jpt* G) { G->X = C->gx; G->Y = C->gy; G->Z = C->p.one; }

/* reduce a 256-bit integer mod n (n > 2^255, so one subtraction suffices) */
static void scalar_reduce(const curve* C, u256* r, const u256* a)
{
    *r = *a;
    if (u256_cmp(r, &C->n_plain) >= 0) u256_sub(r, r, &C->n_plain);
}
/* plain scalar ops mod n through the Montgomery context */
static void scalar_mul(const curve* C, u256* r, const u256* a, const u256* b)
{
    u256 am, bm, t;
    to_mont(&C->n, &am, a);
    to_mont(&C->n, &bm, b);
    mont_mul(&C->n, &t, &am, &bm);
    from_mont(&C->n, r, &t);
}
static void scalar_inv(const curve* C, u256* r, const u256* a)
{
    u256 am, t;
    to_mont(&C->n, &am, a);
    mont_inv(&C->n, &t, &am);
    from_mont(&C->n, r, &t);
}

static void put_pub(uint8_t pub[64], const u256* x, const u256* y)
{
    u256_to_be(pub, x);
    u256_to_be(pub + 32, y);
}

static int pubkey(const curve* C, const uint8_t sk[32], uint8_t pub[64])
{
    u256 d, zero = {{0, 0, 0, 0}}, x, y;
    u256_from_be(&d, sk);
    if (u256_is_zero(&d) || u256_cmp(&d, &C->n_plain) >= 0) return -1;
    jpt G, Q, inf;
    gen_point(C, &G);
    pt_set_inf(&inf);
    pt_mul2(C, &Q, &d, &G, &zero, &inf);
    if (pt_affine(C, &x, &y, &Q)) return -1;
    put_pub(pub, &x, &y);
    return 0;
}

int oracle_secp256k1_pubkey(const uint8_t sk[32], uint8_t pub[64])
{
    ec_init();
    return pubkey(&g_secp, sk, pub);
}
int oracle_sm2_pubkey(const uint8_t sk[32], uint8_t pub[64])
{
    ec_init();
    return pubkey(&g_sm2, sk, pub);
}

/* libsecp256k1 secp256k1_ecdsa_recover (via wedpr_secp256k1_recover_public_key,
 * Secp256k1Crypto.cpp:79-93): parse_compact rejects r,s >= n and recid > 3; recover rejects
 * r == 0, s == 0, (recid&2 and r >= p-n), x not on the curve, Q = infinity. */
int oracle_secp256k1_recover(const uint8_t hash[32], const uint8_t* sig, size_t siglen,
                             uint8_t pub[64])
{
    ec_init();
    const curve* C = &g_secp;
    const mont* f = &C->p;
    if (siglen != 65) return -1; /* SECP256K1_SIGNATURE_LEN (Secp256k1Crypto.h:29); other lengths unpinned */
    int v = sig[64];
    if (v > 3) return -1; /* SignatureTest.cpp:156-162 (v = 4 must throw) */
    u256 r, s, e, x;
    u256_from_be(&r, sig);
    u256_from_be(&s, sig + 32);
    if (u256_cmp(&r, &C->n_plain) >= 0 || u256_cmp(&s, &C->n_plain) >= 0) return -1;
    if (u256_is_zero(&r) || u256_is_zero(&s)) return -1;
    x = r;
    if (v & 2) {
        u256 pmn;
        u256_sub(&pmn, &f->m, &C->n_plain);
        if (u256_cmp(&r, &pmn) >= 0) return -1;
        u256_add(&x, &r, &C->n_plain);
    }
    /* y = sqrt(x^3 + 7) = rhs^((p+1)/4), p = 3 mod 4 */
    u256 xm, rhs, y, ex, one = {{1, 0, 0, 0}}, t;
    to_mont(f, &xm, &x);
    mont_mul(f, &rhs, &xm, &xm);
    mont_mul(f, &rhs, &rhs, &xm);
    mod_add(f, &rhs, &rhs, &C->b);
    u256_add(&ex, &f->m, &one);
    for (int i = 0; i < 4; ++i) ex.v[i] = (ex.v[i] >> 2) | (i < 3 ? ex.v[i + 1] << 62 : 0);
    mont_pow(f, &y, &rhs, &ex);
    mont_mul(f, &t, &y, &y);
    if (u256_cmp(&t, &rhs) != 0) return -1;
    u256 yp;
    from_mont(f, &yp, &y);
    if ((int)(yp.v[0] & 1) != (v & 1)) mod_neg(f, &y, &y);
    jpt R = {xm, y, f->one}, G, Q;
    gen_point(C, &G);
    u256_from_be(&e, hash);
    scalar_reduce(C, &e, &e);
    u256 rinv, u1, u2;
    scalar_inv(C, &rinv, &r);
    scalar_mul(C, &u1, &e, &rinv);
    mod_neg(&C->n, &u1, &u1);
    scalar_mul(C, &u2, &s, &rinv);
    pt_mul2(C, &Q, &u1, &G, &u2, &R);
    u256 qx, qy;
    if (pt_affine(C, &qx, &qy, &Q)) return -1;
    put_pub(pub, &qx, &qy);
    return 0;
}

/* libsecp256k1 secp256k1_ecdsa_sig_sign + low-S normalisation, as wedpr_secp256k1_sign
 * (Secp256k1Crypto.cpp:33-49) produces: recid = (R.x >= n ? 2 : 0) | odd(R.y). */
int oracle_secp256k1_sign(const uint8_t sk[32], const uint8_t hash[32], const uint8_t kb[32],
                          uint8_t sig[65])
{
    ec_init();
    const curve* C = &g_secp;
    u256 d, k, e, zero = {{0, 0, 0, 0}}, rx, ry, r, s, t;
    u256_from_be(&d, sk);
    u256_from_be(&k, kb);
    if (u256_is_zero(&d) || u256_cmp(&d, &C->n_plain) >= 0) return -1;
    if (u256_is_zero(&k) || u256_cmp(&k, &C->n_plain) >= 0) return -1;
    u256_from_be(&e, hash);
    scalar_reduce(C, &e, &e);
    jpt G, Rp, inf;
    gen_point(C, &G);
    pt_set_inf(&inf);
    pt_mul2(C, &Rp, &k, &G, &zero, &inf);
    if (pt_affine(C, &rx, &ry, &Rp)) return -1;
    int recid = (int)(ry.v[0] & 1);
    if (u256_cmp(&rx, &C->n_plain) >= 0) recid |= 2;
    scalar_reduce(C, &r, &rx);
    if (u256_is_zero(&r)) return -1;
    scalar_mul(C, &t, &r, &d);
    mod_add(&C->n, &t, &t, &e);
    u256 kinv;
    scalar_inv(C, &kinv, &k);
    scalar_mul(C, &s, &kinv, &t);
    if (u256_is_zero(&s)) return -1;
    u256 half = C->n_plain; /* n >> 1 */
    for (int i = 0; i < 4; ++i) half.v[i] = (half.v[i] >> 1) | (i < 3 ? half.v[i + 1] << 63 : 0);
    if (u256_cmp(&s, &half) > 0) {
        mod_neg(&C->n, &s, &s);
        recid ^= 1;
    }
    u256_to_be(sig, &r);
    u256_to_be(sig + 32, &s);
    sig[64] = (uint8_t)recid;
    return 0;
}

/* libsecp256k1 secp256k1_ecdsa_verify (rejects high-S) as wedpr_secp256k1_verify
 * (Secp256k1Crypto.cpp:51-63).  Only the first 64 signature bytes are the (r, s) pair. */
int oracle_secp256k1_verify(const uint8_t pub[64], const uint8_t hash[32], const uint8_t* sig,
                            size_t siglen)
{
    ec_init();
    const curve* C = &g_secp;
    if (siglen < 64) return -1;
    u256 px, py, r, s, e, half, w, u1, u2, x, y;
    u256_from_be(&px, pub);
    u256_from_be(&py, pub + 32);
    jpt P, G, Q;
    if (pt_from_affine(C, &P, &px, &py)) return -1;
    u256_from_be(&r, sig);
    u256_from_be(&s, sig + 32);
    if (u256_is_zero(&r) || u256_is_zero(&s)) return -1;
    if (u256_cmp(&r, &C->n_plain) >= 0 || u256_cmp(&s, &C->n_plain) >= 0) return -1;
    half = C->n_plain;
    for (int i = 0; i < 4; ++i) half.v[i] = (half.v[i] >> 1) | (i < 3 ? half.v[i + 1] << 63 : 0);
    if (u256_cmp(&s, &half) > 0) return -1;
    u256_from_be(&e, hash);
    scalar_reduce(C, &e, &e);
    scalar_inv(C, &w, &s);
    scalar_mul(C, &u1, &e, &w);
    scalar_mul(C, &u2, &r, &w);
    gen_point(C, &G);
    pt_mul2(C, &Q, &u1, &G, &u2, &P);
    if (pt_affine(C, &x, &y, &Q)) return -1;
    scalar_reduce(C, &x, &x);
    return u256_cmp(&x, &r) == 0 ? 0 : -1;
}

/* ---------------- SM2 ---------------- */
/* Z_A = SM3(ENTL || ID || a || b || xG || yG || xA || yA), ID = "1234567812345678"
 * (fast_sm2.cpp:34 c_userId, passed to sm2_do_verify at :203) */
void oracle_sm2_za(const uint8_t pub[64], uint8_t za[32])
{
    ec_init();
    const curve* C = &g_sm2;
    uint8_t buf[2 + 16 + 32 * 6];
    u256 t;
    buf[0] = 0x00; buf[1] = 0x80; /* ENTL = 16 bytes * 8 = 128 bits */
    memcpy(buf + 2, "1234567812345678", 16);
    from_mont(&C->p, &t, &C->a); u256_to_be(buf + 18, &t);
    from_mont(&C->p, &t, &C->b); u256_to_be(buf + 50, &t);
    from_mont(&C->p, &t, &C->gx); u256_to_be(buf + 82, &t);
    from_mont(&C->p, &t, &C->gy); u256_to_be(buf + 114, &t);
    memcpy(buf + 146, pub, 64);
    oracle_sm3(buf, sizeof(buf), za);
}

static void sm2_e(const uint8_t pub[64], const uint8_t hash[32], u256* e)
{
    uint8_t m[64], d[32];
    oracle_sm2_za(pub, m);
    memcpy(m + 32, hash, 32);
    oracle_sm3(m, 64, d);
    u256_from_be(e, d);
}

int oracle_sm2_recover(const uint8_t hash[32], const uint8_t* sig, size_t siglen, uint8_t pub[64])
{
    ec_init();
    const curve* C = &g_sm2;
    /* SignatureDataWithPub::decode (SignatureDataWithPub.h:55-64): pub = every byte after r||s;
     * hex2point of "04"||hex(pub) (fast_sm2.cpp:142-160) succeeds only for exactly 64 bytes. */
    if (siglen != 128) return -1;
    u256 px, py, r, s, e, t, x, y;
    u256_from_be(&px, sig + 64);
    u256_from_be(&py, sig + 96);
    jpt P, G, Q;
    if (pt_from_affine(C, &P, &px, &py)) return -1; /* oct2point: x,y < p and on the curve */
    u256_from_be(&r, sig);
    u256_from_be(&s, sig + 32);
    if (u256_is_zero(&r) || u256_is_zero(&s)) return -1;
    if (u256_cmp(&r, &C->n_plain) >= 0 || u256_cmp(&s, &C->n_plain) >= 0) return -1;
    sm2_e(sig + 64, hash, &e);
    mod_add(&C->n, &t, &r, &s); /* t = (r + s) mod n */
    if (u256_is_zero(&t)) return -1;
    gen_point(C, &G);
    pt_mul2(C, &Q, &s, &G, &t, &P);
    if (pt_affine(C, &x, &y, &Q)) return -1;
    /* R = (e + x1) mod n ; accept iff R == r.  e and x1 may exceed n: reduce both first. */
    scalar_reduce(C, &e, &e);
    scalar_reduce(C, &x, &x);
    mod_add(&C->n, &t, &e, &x);
    if (u256_cmp(&t, &r) != 0) return -1;
    if (pub) memcpy(pub, sig + 64, 64);
    return 0;
}

/* GB/T 32918.2 signature generation with an explicit nonce (SM2Crypto::sign, SM2Crypto.cpp:40-64
 * appends the public key to r||s when _signatureWithPub). */
int oracle_sm2_sign(const uint8_t sk[32], const uint8_t hash[32], const uint8_t kb[32],
                    uint8_t sig[128])
{
    ec_init();
    const curve* C = &g_sm2;
    uint8_t pub[64];
    u256 d, k, e, x1, y1, r, s, t, zero = {{0, 0, 0, 0}}, one = {{1, 0, 0, 0}};
    u256_from_be(&d, sk);
    u256_from_be(&k, kb);
    if (u256_is_zero(&k) || u256_cmp(&k, &C->n_plain) >= 0) return -1;
    u256 nm1;
    u256_sub(&nm1, &C->n_plain, &one);
    if (u256_is_zero(&d) || u256_cmp(&d, &nm1) >= 0) return -1; /* d in [1, n-2] */
    if (pubkey(C, sk, pub)) return -1;
    sm2_e(pub, hash, &e);
    scalar_reduce(C, &e, &e);
    jpt G, K, inf;
    gen_point(C, &G);
    pt_set_inf(&inf);
    pt_mul2(C, &K, &k, &G, &zero, &inf);
    if (pt_affine(C, &x1, &y1, &K)) return -1;
    scalar_reduce(C, &x1, &x1);
    mod_add(&C->n, &r, &e, &x1);
    if (u256_is_zero(&r)) return -1;
    mod_add(&C->n, &t, &r, &k);
    if (u256_is_zero(&t)) return -1;
    u256 dp1, inv, rd;
    mod_add(&C->n, &dp1, &d, &one);
    scalar_inv(C, &inv, &dp1);
    scalar_mul(C, &rd, &r, &d);
    mod_sub(&C->n, &t, &k, &rd);
    scalar_mul(C, &s, &inv, &t);
    if (u256_is_zero(&s)) return -1;
    u256_to_be(sig, &r);
    u256_to_be(sig + 32, &s);
    memcpy(sig + 64, pub, 64);
    return 0;
}
