// hash_device.h -- device-side Keccak-256 and SM3 for gfx950 (one message per lane).
//
// Replaces bcos::crypto::hasher::openssl::OpenSSLHasher<Keccak256|SM3>
// (bcos-crypto/bcos-crypto/hasher/OpenSSLHasher.h:22-143; Keccak pad byte 0x01 per :51-80;
// SM3 via EVP_sm3 :113-116).  Integer-ALU work: Keccak-f[1600] on 64-bit lanes that the compiler
// lowers to 32-bit v_xor3 / v_alignbit / v_bfi pairs; SM3 on 32-bit words.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bcosgpu {

enum Hasher : int { KECCAK256 = 0, SM3 = 1 };

// ------------------------------------------------------------------ message readers
// Reads the little-endian 32-bit word i (bytes 4i..4i+3) of a byte string of length len that
// starts at an arbitrary address; bytes past len read as zero.  Only aligned dwords that contain
// at least one message byte are loaded, so a read never leaves the pages holding the message.
struct ByteReader {
    const uint32_t* q;  // aligned base
    uint32_t sh;        // misalignment in bytes (0..3)
    uint32_t len;       // message length in bytes
    uint32_t nq;        // number of aligned dwords overlapping the message
    __device__ ByteReader(const uint8_t* p, uint32_t n) {
        uintptr_t a = reinterpret_cast<uintptr_t>(p);
        sh = static_cast<uint32_t>(a & 3u);
        q = reinterpret_cast<const uint32_t*>(a - sh);
        len = n;
        nq = (n + sh + 3u) >> 2;
    }
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        uint32_t lo = i < nq ? q[i] : 0u;
        uint32_t hi = (i + 1u) < nq ? q[i + 1u] : 0u;
        uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, sh);
        uint32_t b = i * 4u;
        if (b + 4u > len) w = b >= len ? 0u : (w & ((1u << ((len - b) * 8u)) - 1u));
        return w;
    }
};

// Reader for 4-byte-aligned messages whose length is a multiple of 4 (Merkle nodes: 32-B children).
struct AlignedReader {
    const uint32_t* q;
    uint32_t len;
    uint32_t nw;
    __device__ AlignedReader(const uint8_t* p, uint32_t n)
        : q(reinterpret_cast<const uint32_t*>(p)), len(n), nw(n >> 2) {}
    __device__ __forceinline__ uint32_t word(uint32_t i) const { return i < nw ? q[i] : 0u; }
};

// ------------------------------------------------------------------ Keccak-256
__device__ __constant__ static const uint64_t kKeccakRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
    return (x << r) | (x >> (64 - r));
}

// Keccak-f[1600], fully unrolled; state lane index x + 5y.
__device__ __forceinline__ void keccak_f1600(uint64_t s[25]) {
#pragma unroll 1
    for (int round = 0; round < 24; ++round) {
        uint64_t c0 = s[0] ^ s[5] ^ s[10] ^ s[15] ^ s[20];
        uint64_t c1 = s[1] ^ s[6] ^ s[11] ^ s[16] ^ s[21];
        uint64_t c2 = s[2] ^ s[7] ^ s[12] ^ s[17] ^ s[22];
        uint64_t c3 = s[3] ^ s[8] ^ s[13] ^ s[18] ^ s[23];
        uint64_t c4 = s[4] ^ s[9] ^ s[14] ^ s[19] ^ s[24];
        uint64_t d0 = c4 ^ rotl64(c1, 1), d1 = c0 ^ rotl64(c2, 1), d2 = c1 ^ rotl64(c3, 1),
                 d3 = c2 ^ rotl64(c4, 1), d4 = c3 ^ rotl64(c0, 1);
        // theta + rho + pi: b[y + 5((2x+3y)%5)] = rotl(a[x+5y] ^ d[x], r[x][y])
        uint64_t b0 = s[0] ^ d0;
        uint64_t b10 = rotl64(s[1] ^ d1, 1);
        uint64_t b20 = rotl64(s[2] ^ d2, 62);
        uint64_t b5 = rotl64(s[3] ^ d3, 28);
        uint64_t b15 = rotl64(s[4] ^ d4, 27);
        uint64_t b16 = rotl64(s[5] ^ d0, 36);
        uint64_t b1 = rotl64(s[6] ^ d1, 44);
        uint64_t b11 = rotl64(s[7] ^ d2, 6);
        uint64_t b21 = rotl64(s[8] ^ d3, 55);
        uint64_t b6 = rotl64(s[9] ^ d4, 20);
        uint64_t b7 = rotl64(s[10] ^ d0, 3);
        uint64_t b17 = rotl64(s[11] ^ d1, 10);
        uint64_t b2 = rotl64(s[12] ^ d2, 43);
        uint64_t b12 = rotl64(s[13] ^ d3, 25);
        uint64_t b22 = rotl64(s[14] ^ d4, 39);
        uint64_t b23 = rotl64(s[15] ^ d0, 41);
        uint64_t b8 = rotl64(s[16] ^ d1, 45);
        uint64_t b18 = rotl64(s[17] ^ d2, 15);
        uint64_t b3 = rotl64(s[18] ^ d3, 21);
        uint64_t b13 = rotl64(s[19] ^ d4, 8);
        uint64_t b14 = rotl64(s[20] ^ d0, 18);
        uint64_t b24 = rotl64(s[21] ^ d1, 2);
        uint64_t b9 = rotl64(s[22] ^ d2, 61);
        uint64_t b19 = rotl64(s[23] ^ d3, 56);
        uint64_t b4 = rotl64(s[24] ^ d4, 14);
        // chi + iota
        s[0] = b0 ^ (~b1 & b2) ^ kKeccakRC[round];
        s[1] = b1 ^ (~b2 & b3);
        s[2] = b2 ^ (~b3 & b4);
        s[3] = b3 ^ (~b4 & b0);
        s[4] = b4 ^ (~b0 & b1);
        s[5] = b5 ^ (~b6 & b7);
        s[6] = b6 ^ (~b7 & b8);
        s[7] = b7 ^ (~b8 & b9);
        s[8] = b8 ^ (~b9 & b5);
        s[9] = b9 ^ (~b5 & b6);
        s[10] = b10 ^ (~b11 & b12);
        s[11] = b11 ^ (~b12 & b13);
        s[12] = b12 ^ (~b13 & b14);
        s[13] = b13 ^ (~b14 & b10);
        s[14] = b14 ^ (~b10 & b11);
        s[15] = b15 ^ (~b16 & b17);
        s[16] = b16 ^ (~b17 & b18);
        s[17] = b17 ^ (~b18 & b19);
        s[18] = b18 ^ (~b19 & b15);
        s[19] = b19 ^ (~b15 & b16);
        s[20] = b20 ^ (~b21 & b22);
        s[21] = b21 ^ (~b22 & b23);
        s[22] = b22 ^ (~b23 & b24);
        s[23] = b23 ^ (~b24 & b20);
        s[24] = b24 ^ (~b20 & b21);
    }
}

// Keccak-256 of a whole message through a reader (rate 136 B = 34 words, pad 0x01 ... 0x80).
template <class Reader>
__device__ __forceinline__ void keccak256_msg(const Reader& rd, uint32_t len, uint32_t out[8]) {
    uint64_t s[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = 0;
    const uint32_t nblocks = len / 136u + 1u;  // padding always fits in the final block
    const uint32_t padw = len >> 2, padb = (len & 3u) * 8u;
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        const uint32_t w0 = blk * 34u;
#pragma unroll
        for (int j = 0; j < 17; ++j) {
            uint32_t lo = rd.word(w0 + 2 * j), hi = rd.word(w0 + 2 * j + 1);
            if (w0 + 2 * j == padw) lo ^= 1u << padb;
            if (w0 + 2 * j + 1 == padw) hi ^= 1u << padb;
            s[j] ^= (static_cast<uint64_t>(hi) << 32) | lo;
        }
        if (blk + 1 == nblocks) s[16] ^= 0x8000000000000000ULL;
        keccak_f1600(s);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out[2 * i] = static_cast<uint32_t>(s[i]);
        out[2 * i + 1] = static_cast<uint32_t>(s[i] >> 32);
    }
}

// Keccak-256 of exactly 64 bytes held in registers (pubkey X||Y as little-endian words) -- the
// address hash right160(Keccak256(pub)) (KeyPair.h:30-33).
__device__ __forceinline__ void keccak256_64(const uint32_t m[16], uint32_t out[8]) {
    uint64_t s[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = (static_cast<uint64_t>(m[2 * j + 1]) << 32) | m[2 * j];
    s[8] = 1;
    s[16] = 0x8000000000000000ULL;
    keccak_f1600(s);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out[2 * i] = static_cast<uint32_t>(s[i]);
        out[2 * i + 1] = static_cast<uint32_t>(s[i] >> 32);
    }
}

// ------------------------------------------------------------------ SM3 (GB/T 32905-2016)
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) {
    return __builtin_amdgcn_alignbit(x, x, (32 - r) & 31);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t sm3_p0(uint32_t x) { return x ^ rotl32(x, 9) ^ rotl32(x, 17); }
__device__ __forceinline__ uint32_t sm3_p1(uint32_t x) { return x ^ rotl32(x, 15) ^ rotl32(x, 23); }

__device__ __forceinline__ void sm3_init(uint32_t V[8]) {
    V[0] = 0x7380166fu; V[1] = 0x4914b2b9u; V[2] = 0x172442d7u; V[3] = 0xda8a0600u;
    V[4] = 0xa96f30bcu; V[5] = 0x163138aau; V[6] = 0xe38dee4du; V[7] = 0xb0fb0e4eu;
}

// One compression; W[0..15] are the block's big-endian words.  Message expansion is computed on
// the fly in a 16-word ring so only 16 words stay live.
__device__ __forceinline__ void sm3_compress(uint32_t V[8], uint32_t W[16]) {
    uint32_t A = V[0], B = V[1], C = V[2], D = V[3], E = V[4], F = V[5], G = V[6], H = V[7];
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        // W[j+4] is needed for W'[j] = W[j] ^ W[j+4]
        if (j >= 12) {
            const int t = j + 4;  // expand W[t], t in [16, 68)
            uint32_t x = W[(t - 16) & 15] ^ W[(t - 9) & 15] ^ rotl32(W[(t - 3) & 15], 15);
            W[t & 15] = sm3_p1(x) ^ rotl32(W[(t - 13) & 15], 7) ^ W[(t - 6) & 15];
        }
        const uint32_t wj = W[j & 15], wj4 = W[(j + 4) & 15];
        const uint32_t T = j < 16 ? 0x79cc4519u : 0x7a879d8au;
        const uint32_t a12 = rotl32(A, 12);
        const uint32_t SS1 = rotl32(a12 + E + rotl32(T, j & 31), 7);
        const uint32_t SS2 = SS1 ^ a12;
        const uint32_t FF = j < 16 ? (A ^ B ^ C) : ((A & B) | (A & C) | (B & C));
        const uint32_t GG = j < 16 ? (E ^ F ^ G) : ((E & F) | (~E & G));
        const uint32_t TT1 = FF + D + SS2 + (wj ^ wj4);
        const uint32_t TT2 = GG + H + SS1 + wj;
        D = C; C = rotl32(B, 9); B = A; A = TT1;
        H = G; G = rotl32(F, 19); F = E; E = sm3_p0(TT2);
    }
    V[0] ^= A; V[1] ^= B; V[2] ^= C; V[3] ^= D; V[4] ^= E; V[5] ^= F; V[6] ^= G; V[7] ^= H;
}

// SM3 of a whole message through a reader; out[] holds the digest as big-endian words.
template <class Reader>
__device__ __forceinline__ void sm3_msg(const Reader& rd, uint32_t len, uint32_t out[8]) {
    uint32_t V[8];
    sm3_init(V);
    const uint32_t nblocks = (len + 8u) / 64u + 1u;
    const uint32_t padw = len >> 2, padb = 24u - (len & 3u) * 8u;
    const uint64_t bits = static_cast<uint64_t>(len) * 8u;
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        uint32_t W[16];
        const uint32_t w0 = blk * 16u;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t w = bswap32(rd.word(w0 + j));
            if (w0 + j == padw) w ^= 0x80u << padb;
            W[j] = w;
        }
        if (blk + 1 == nblocks) {
            W[14] = static_cast<uint32_t>(bits >> 32);
            W[15] = static_cast<uint32_t>(bits);
        }
        sm3_compress(V, W);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = V[i];
}

// SM3 of exactly 64 bytes given as big-endian words (pubkey address hash).
__device__ __forceinline__ void sm3_64(const uint32_t m_be[16], uint32_t out[8]) {
    uint32_t V[8], W[16];
    sm3_init(V);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = m_be[j];
    sm3_compress(V, W);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = 0;
    W[0] = 0x80000000u;
    W[15] = 512u;
    sm3_compress(V, W);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = V[i];
}

// Store a 32-byte digest.  Keccak words are little-endian lanes (byte order == memory order);
// SM3 words are big-endian.
__device__ __forceinline__ void store_digest(int hasher, uint8_t* dst, const uint32_t d[8]) {
    uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = hasher == SM3 ? bswap32(d[i]) : d[i];
}

}  // namespace bcosgpu
