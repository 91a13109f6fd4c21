/*
 * hash.c -- oracle restatement of the two hashers on the path.  TEST INFRASTRUCTURE ONLY.
 *
 * Keccak256: the reference hashes with an OpenSSL SHA3-256 context whose pad byte is patched from
 *   0x06 to 0x01 (bcos-crypto/bcos-crypto/hasher/OpenSSLHasher.h:51-80): i.e. original Keccak
 *   padding (0x01 ... 0x80), rate 136 B, 256-bit output.  Restated from the Keccak-f[1600] spec.
 * SM3: EVP_sm3 (OpenSSLHasher.h:113-116), restated from GB/T 32905-2016.
 * Pinned by bcos-crypto/test/unittests/HashTest.cpp:59-99 (tests/golden/kat.json).
 */
#include "oracle.h"
#include <string.h>

static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
/* rho offsets indexed by lane x + 5y */
static const int KRHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline uint64_t rol64(uint64_t x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }

/* Keccak-f[1600]: theta, rho+pi, chi, iota -- written from the specification's definitions */
static void keccak_f1600(uint64_t A[25])
{
    for (int round = 0; round < 24; ++round) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        /* B[y, 2x+3y] = rot(A[x,y], r[x,y]) */
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(A[x + 5 * y], KRHO[x + 5 * y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= KRC[round];
    }
}

void oracle_keccak256(const uint8_t* in, size_t len, uint8_t out[32])
{
    enum { RATE = 136 };
    uint64_t A[25];
    memset(A, 0, sizeof(A));
    uint8_t block[RATE];
    size_t off = 0;
    for (;;) {
        size_t take = len - off;
        int last = take < RATE;
        if (!last) take = RATE;
        memset(block, 0, RATE);
        memcpy(block, in + off, take);
        if (last) { /* multi-rate padding with the Keccak domain byte 0x01 */
            block[take] ^= 0x01;
            block[RATE - 1] ^= 0x80;
        }
        for (int i = 0; i < RATE / 8; ++i) {
            uint64_t w = 0;
            for (int b = 7; b >= 0; --b) w = (w << 8) | block[8 * i + b]; /* little-endian lanes */
            A[i] ^= w;
        }
        keccak_f1600(A);
        off += take;
        if (last) break;
    }
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(A[i] >> (8 * b));
}

/* ---------------- SM3 (GB/T 32905-2016) ---------------- */
static inline uint32_t rol32(uint32_t x, int r) { r &= 31; return r ? (x << r) | (x >> (32 - r)) : x; }
static inline uint32_t sm3_p0(uint32_t x) { return x ^ rol32(x, 9) ^ rol32(x, 17); }
static inline uint32_t sm3_p1(uint32_t x) { return x ^ rol32(x, 15) ^ rol32(x, 23); }

static void sm3_compress(uint32_t V[8], const uint8_t blk[64])
{
    uint32_t W[68], W1[64];
    for (int j = 0; j < 16; ++j)
        W[j] = ((uint32_t)blk[4 * j] << 24) | ((uint32_t)blk[4 * j + 1] << 16) |
               ((uint32_t)blk[4 * j + 2] << 8) | blk[4 * j + 3];
    for (int j = 16; j < 68; ++j)
        W[j] = sm3_p1(W[j - 16] ^ W[j - 9] ^ rol32(W[j - 3], 15)) ^ rol32(W[j - 13], 7) ^ W[j - 6];
    for (int j = 0; j < 64; ++j) W1[j] = W[j] ^ W[j + 4];
    uint32_t A = V[0], B = V[1], C = V[2], D = V[3], E = V[4], F = V[5], G = V[6], H = V[7];
    for (int j = 0; j < 64; ++j) {
        uint32_t T = j < 16 ? 0x79cc4519u : 0x7a879d8au;
        uint32_t SS1 = rol32(rol32(A, 12) + E + rol32(T, j), 7);
        uint32_t SS2 = SS1 ^ rol32(A, 12);
        uint32_t FF = j < 16 ? (A ^ B ^ C) : ((A & B) | (A & C) | (B & C));
        uint32_t GG = j < 16 ? (E ^ F ^ G) : ((E & F) | (~E & G));
        uint32_t TT1 = FF + D + SS2 + W1[j];
        uint32_t TT2 = GG + H + SS1 + W[j];
        D = C; C = rol32(B, 9); B = A; A = TT1;
        H = G; G = rol32(F, 19); F = E; E = sm3_p0(TT2);
    }
    V[0] ^= A; V[1] ^= B; V[2] ^= C; V[3] ^= D; V[4] ^= E; V[5] ^= F; V[6] ^= G; V[7] ^= H;
}

void oracle_sm3(const uint8_t* in, size_t len, uint8_t out[32])
{
    uint32_t V[8] = {0x7380166f, 0x4914b2b9, 0x172442d7, 0xda8a0600,
                     0xa96f30bc, 0x163138aa, 0xe38dee4d, 0xb0fb0e4e};
    size_t full = len / 64;
    for (size_t i = 0; i < full; ++i) sm3_compress(V, in + 64 * i);
    uint8_t tail[128];
    size_t rem = len - 64 * full;
    memset(tail, 0, sizeof(tail));
    memcpy(tail, in + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tl = rem + 1 + 8 <= 64 ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int b = 0; b < 8; ++b) tail[tl - 1 - b] = (uint8_t)(bits >> (8 * b));
    sm3_compress(V, tail);
    if (tl == 128) sm3_compress(V, tail + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(V[i] >> 24); out[4 * i + 1] = (uint8_t)(V[i] >> 16);
        out[4 * i + 2] = (uint8_t)(V[i] >> 8); out[4 * i + 3] = (uint8_t)V[i];
    }
}

void oracle_hash(int hasher, const uint8_t* in, size_t len, uint8_t out[32])
{
    if (hasher == ORACLE_SM3) oracle_sm3(in, len, out);
    else oracle_keccak256(in, len, out);
}
