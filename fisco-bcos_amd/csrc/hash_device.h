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

// ByteReader without branches (hash_batch_kernel): both dwords of a word are loaded from clamped
// indices and selected, so a block's loads issue back to back under one wait instead of one branch
// and one s_waitcnt each.  Still never reads a dword outside the message: an empty message that
// overlaps no dword reads a zero constant.
__device__ __constant__ static const uint32_t kZeroDwords[2] = {0u, 0u};
struct FlatReader {
    const uint32_t* q;  // aligned base (kZeroDwords when no dword overlaps the message)
    uint32_t sh, len, nq, last;
    __device__ FlatReader(const uint8_t* p, uint32_t n) {
        uintptr_t a = reinterpret_cast<uintptr_t>(p);
        sh = static_cast<uint32_t>(a & 3u);
        nq = (n + sh + 3u) >> 2;
        q = nq ? reinterpret_cast<const uint32_t*>(a - sh) : kZeroDwords;
        last = nq ? nq - 1u : 0u;
        len = n;
    }
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        const uint32_t l = q[i < last ? i : last], h = q[i + 1u < last ? i + 1u : last];
        const uint32_t lo = i < nq ? l : 0u, hi = i + 1u < nq ? h : 0u;
        uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, sh);
        const uint32_t b = i * 4u;
        const uint32_t keep = b >= len ? 0u : b + 4u > len ? (1u << ((len - b) * 8u)) - 1u : 0xffffffffu;
        return w & keep;
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

// AlignedReader for messages of at least 4 bytes (Merkle nodes: 32 B per child): every word is loaded
// from a clamped index (the last message word past the end) and selected, so a block's sixteen loads
// carry no branches and issue back to back under one wait, where AlignedReader's guarded loads each
// sit in their own branch behind their own s_waitcnt.
struct NodeReader {
    const uint32_t* q;
    uint32_t nw;  // >= 1
    __device__ NodeReader(const uint8_t* p, uint32_t n) : q(reinterpret_cast<const uint32_t*>(p)), nw(n >> 2) {}
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        const uint32_t w = q[i < nw ? i : nw - 1u];
        return i < nw ? w : 0u;
    }
};

// ------------------------------------------------------------------ Keccak-256
__device__ __constant__ static const uint64_t kKeccakRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

// Keccak-f[1600] on 32-bit halves (gfx950 has no 64-bit logic ops): theta folds into 3-input
// v_bitop3 XORs (column parity: 2 per half; a ^ C[x-1] ^ rotl1(C[x+1]) in one), rho is a v_alignbit
// pair, chi is one v_bitop3 (a ^ (~b & c)) per half -- ~180 VALU per round.  State lane x + 5y.
struct KLane {
    uint32_t lo, hi;
};
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t chi32(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xD2);  // a ^ (~b & c)
}
template <int R>
__device__ __forceinline__ KLane rotl_lane(KLane x) {
    if constexpr (R == 0) {
        return x;
    } else if constexpr (R < 32) {
        return {__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - R), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - R)};
    } else if constexpr (R == 32) {
        return {x.hi, x.lo};
    } else {
        return {__builtin_amdgcn_alignbit(x.hi, x.lo, 64 - R), __builtin_amdgcn_alignbit(x.lo, x.hi, 64 - R)};
    }
}

__device__ __forceinline__ void keccak_f1600(uint64_t s[25]) {
    KLane a[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = {static_cast<uint32_t>(s[i]), static_cast<uint32_t>(s[i] >> 32)};
#pragma unroll 1
    for (int round = 0; round < 24; ++round) {
        KLane c[5], e[5], b[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            c[x].lo = xor3(xor3(a[x].lo, a[x + 5].lo, a[x + 10].lo), a[x + 15].lo, a[x + 20].lo);
            c[x].hi = xor3(xor3(a[x].hi, a[x + 5].hi, a[x + 10].hi), a[x + 15].hi, a[x + 20].hi);
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) e[x] = rotl_lane<1>(c[(x + 1) % 5]);
        // theta + rho + pi: b[y + 5((2x+3y)%5)] = rotl(a[x+5y] ^ C[x-1] ^ rotl1(C[x+1]), r[x][y])
#define KECCAK_TRP(SRC, R, DST, XM1, X) \
    b[DST] = rotl_lane<R>(KLane{xor3(a[SRC].lo, c[XM1].lo, e[X].lo), xor3(a[SRC].hi, c[XM1].hi, e[X].hi)})
        KECCAK_TRP(0, 0, 0, 4, 0);
        KECCAK_TRP(1, 1, 10, 0, 1);
        KECCAK_TRP(2, 62, 20, 1, 2);
        KECCAK_TRP(3, 28, 5, 2, 3);
        KECCAK_TRP(4, 27, 15, 3, 4);
        KECCAK_TRP(5, 36, 16, 4, 0);
        KECCAK_TRP(6, 44, 1, 0, 1);
        KECCAK_TRP(7, 6, 11, 1, 2);
        KECCAK_TRP(8, 55, 21, 2, 3);
        KECCAK_TRP(9, 20, 6, 3, 4);
        KECCAK_TRP(10, 3, 7, 4, 0);
        KECCAK_TRP(11, 10, 17, 0, 1);
        KECCAK_TRP(12, 43, 2, 1, 2);
        KECCAK_TRP(13, 25, 12, 2, 3);
        KECCAK_TRP(14, 39, 22, 3, 4);
        KECCAK_TRP(15, 41, 23, 4, 0);
        KECCAK_TRP(16, 45, 8, 0, 1);
        KECCAK_TRP(17, 15, 18, 1, 2);
        KECCAK_TRP(18, 21, 3, 2, 3);
        KECCAK_TRP(19, 8, 13, 3, 4);
        KECCAK_TRP(20, 18, 14, 4, 0);
        KECCAK_TRP(21, 2, 24, 0, 1);
        KECCAK_TRP(22, 61, 9, 1, 2);
        KECCAK_TRP(23, 56, 19, 2, 3);
        KECCAK_TRP(24, 14, 4, 3, 4);
#undef KECCAK_TRP
        // chi + iota
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
#pragma unroll
            for (int x = 0; x < 5; ++x) {
                const KLane p = b[y + x], q = b[y + (x + 1) % 5], r = b[y + (x + 2) % 5];
                a[y + x] = {chi32(p.lo, q.lo, r.lo), chi32(p.hi, q.hi, r.hi)};
            }
        }
        const uint64_t rc = kKeccakRC[round];
        a[0].lo ^= static_cast<uint32_t>(rc);
        a[0].hi ^= static_cast<uint32_t>(rc >> 32);
    }
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = (static_cast<uint64_t>(a[i].hi) << 32) | a[i].lo;
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
__device__ __forceinline__ uint32_t sm3_p0(uint32_t x) { return xor3(x, rotl32(x, 9), rotl32(x, 17)); }
__device__ __forceinline__ uint32_t sm3_p1(uint32_t x) { return xor3(x, rotl32(x, 15), rotl32(x, 23)); }

__device__ __forceinline__ void sm3_init(uint32_t V[8]) {
    V[0] = 0x7380166fu; V[1] = 0x4914b2b9u; V[2] = 0x172442d7u; V[3] = 0xda8a0600u;
    V[4] = 0xa96f30bcu; V[5] = 0x163138aau; V[6] = 0xe38dee4du; V[7] = 0xb0fb0e4eu;
}

// One compression; W[0..15] are the block's big-endian words.  Message expansion is computed on
// the fly in a 16-word ring so only 16 words stay live.
template <bool LOW>  // rounds 0..15 (xor FF/GG) or 16..63 (majority / choose)
__device__ __forceinline__ void sm3_round(int j, uint32_t W[16], uint32_t& A, uint32_t& B, uint32_t& C, uint32_t& D,
                                          uint32_t& E, uint32_t& F, uint32_t& G, uint32_t& H) {
    // W[j+4] is needed for W'[j] = W[j] ^ W[j+4]
    if (j >= 12) {
        const int t = j + 4;  // expand W[t], t in [16, 68)
        const uint32_t x = xor3(W[(t - 16) & 15], W[(t - 9) & 15], rotl32(W[(t - 3) & 15], 15));
        W[t & 15] = xor3(sm3_p1(x), rotl32(W[(t - 13) & 15], 7), W[(t - 6) & 15]);
    }
    const uint32_t wj = W[j & 15], wj4 = W[(j + 4) & 15];
    const uint32_t T = LOW ? 0x79cc4519u : 0x7a879d8au;
    const uint32_t a12 = rotl32(A, 12);
    const uint32_t SS1 = rotl32(a12 + E + rotl32(T, j & 31), 7);
    const uint32_t SS2 = SS1 ^ a12;
    // FF: xor / majority, GG: xor / choose -- one v_bitop3 each
    const uint32_t FF = __builtin_amdgcn_bitop3_b32(A, B, C, LOW ? 0x96 : 0xE8);
    const uint32_t GG = __builtin_amdgcn_bitop3_b32(E, F, G, LOW ? 0x96 : 0xCA);
    const uint32_t TT1 = FF + D + SS2 + (wj ^ wj4);
    const uint32_t TT2 = GG + H + SS1 + wj;
    D = C; C = rotl32(B, 9); B = A; A = TT1;
    H = G; G = rotl32(F, 19); F = E; E = sm3_p0(TT2);
}

__device__ __forceinline__ void sm3_compress(uint32_t V[8], uint32_t W[16]) {
    uint32_t A = V[0], B = V[1], C = V[2], D = V[3], E = V[4], F = V[5], G = V[6], H = V[7];
#pragma unroll
    for (int j = 0; j < 16; ++j) sm3_round<true>(j, W, A, B, C, D, E, F, G, H);
#pragma unroll
    for (int j = 16; j < 64; ++j) sm3_round<false>(j, W, A, B, C, D, E, F, G, H);
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

// ------------------------------------------------------------------ lane-cooperative Keccak-256
// For latency-bound hashing (the top levels of a Merkle tree: one 512-byte width-16 node is 4 serial
// permutations), one state is spread over 25 lanes of a 32-lane group, each lane holding one
// A[x][y] as two 32-bit halves; a wave runs two states.  Lanes are placed so that every 5-lane plane
// y sits inside one 16-lane DPP row: row 0 of the group holds y = 0, 1, 2 (lanes 5y + x), row 1 holds
// y = 3, 4 (lanes 16 + 5(y - 3) + x); lanes 15 and 26..31 are idle.  Then a round needs one LDS
// round trip (pi's gather, ds_bpermute) and everything else is DPP row shifts, v_permlane16_swap
// (row 0 <-> row 1) and per-lane selects:
//   theta: t = A ^ A(y+1); plane y = 0 gets C[x] = t ^ A(y+2) ^ t(row 1) (permlane16_swap);
//          D[x] = C[x-1] ^ rotl1(C[x+1]) on plane 0 (row shifts by 1 / 4 within the plane), then
//          broadcast to planes 1, 2 (row_shr 5 / 10) and to row 1 (permlane16_swap)
//   rho: per-lane rotation; pi: one ds_bpermute; chi: A(x+1), A(x+2) by row shifts within the plane
// ~60 VALU per round per lane against ~180 in one lane, and one LDS latency instead of four (the
// previous ds_bpermute-only version: theta's column and neighbour gathers, pi, chi's row gathers).
// Both 32-lane groups of the wave must call it together (DPP and ds_bpermute are wave-wide).
struct KeccakCoop {
    int gl;            // Keccak lane index x + 5y of this lane, >= 25 on idle lanes
    int x, y;          // its position (idle lanes: x = 0, y = 0)
    int pisrc;         // pi: bpermute byte address of the source lane of this lane's B position
    uint32_t sh;       // rho: 32 - (r mod 32), 0 when r mod 32 == 0
    bool swap;         // rho: swap the halves first (see the constructor)
    uint32_t m0;       // all-ones on lane (0, 0) (iota)
    __device__ static int lane_of(int base, int xx, int yy) {
        return base + (yy < 3 ? 5 * yy + xx : 16 + 5 * (yy - 3) + xx);
    }
    __device__ KeccakCoop() {
        const int lane = static_cast<int>(__lane_id());
        const int g = lane & 31, base = lane & 32;
        const bool row0 = g < 15, row1 = g >= 16 && g < 26;
        x = row0 ? g % 5 : row1 ? (g - 16) % 5 : 0;
        y = row0 ? g / 5 : row1 ? 3 + (g - 16) / 5 : 0;
        gl = row0 || row1 ? x + 5 * y : 31;
        // destination (X, Y) = (x, y) of this lane takes source (x', y') with y' = X, 2x' + 3y' = Y (mod 5)
        const int sx = ((3 * (y - 3 * x)) % 5 + 5) % 5;
        pisrc = lane_of(base, sx, x) * 4;
        constexpr uint8_t R[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                   25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
        // rotl(r) of the (lo, hi) pair = two v_alignbit by 32 - (r mod 32) after swapping the halves when
        // r >= 32; when r mod 32 == 0 the shift is 0, where alignbit(p, q, 0) = q, so the halves are
        // swapped once more instead (no branch on the per-lane amount)
        const int r = R[gl < 25 ? gl : 0];
        swap = (r >= 32) != ((r & 31) == 0);
        sh = (r & 31) ? 32u - (r & 31) : 0u;
        m0 = gl == 0 ? 0xffffffffu : 0u;
    }
    template <int CTRL>
    __device__ __forceinline__ static uint32_t dpp(uint32_t v) {
        return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, true));
    }
    // row_shl:k = the value of lane i + k, row_shr:k = of lane i - k (inside the 16-lane row)
    static constexpr int kR1 = 0x101, kR2 = 0x102, kR5 = 0x105, kR10 = 0x10a, kR4 = 0x104;
    static constexpr int kL1 = 0x111, kL3 = 0x113, kL4 = 0x114, kL5 = 0x115, kL10 = 0x11a;
    __device__ __forceinline__ static uint32_t sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }
    __device__ __forceinline__ static uint32_t from_row1(uint32_t v) {  // row 0 lanes read lane + 16
        return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1];
    }
    __device__ __forceinline__ static uint32_t from_row0(uint32_t v) {  // row 1 lanes read lane - 16
        return __builtin_amdgcn_permlane16_swap(v, v, false, false)[0];
    }
    // column parity C[x] (valid on plane y = 0)
    __device__ __forceinline__ static uint32_t colpar(uint32_t a) {
        const uint32_t t = a ^ dpp<kR5>(a);
        return xor3(t, dpp<kR10>(a), from_row1(t));
    }
    __device__ __forceinline__ void permute(uint32_t& lo, uint32_t& hi) const {
        const bool x0 = x == 0, x4 = x == 4, x34 = x >= 3, y1 = y == 1, y2 = y == 2, ry = y >= 3;
#pragma unroll
        for (int round = 0; round < 24; ++round) {
            // theta
            // (every cross-lane fetch is evaluated on all lanes, then selected: a fetch inside one arm
            // of a conditional would run under a partial EXEC and read inactive lanes)
            const uint32_t c_lo = colpar(lo), c_hi = colpar(hi);
            const uint32_t m_lo = sel(x0, dpp<kR4>(c_lo), dpp<kL1>(c_lo));
            const uint32_t m_hi = sel(x0, dpp<kR4>(c_hi), dpp<kL1>(c_hi));
            const uint32_t p_lo = sel(x4, dpp<kL4>(c_lo), dpp<kR1>(c_lo));
            const uint32_t p_hi = sel(x4, dpp<kL4>(c_hi), dpp<kR1>(c_hi));
            uint32_t d_lo = m_lo ^ __builtin_amdgcn_alignbit(p_lo, p_hi, 31);
            uint32_t d_hi = m_hi ^ __builtin_amdgcn_alignbit(p_hi, p_lo, 31);
            d_lo = sel(y1, dpp<kL5>(d_lo), sel(y2, dpp<kL10>(d_lo), d_lo));
            d_hi = sel(y1, dpp<kL5>(d_hi), sel(y2, dpp<kL10>(d_hi), d_hi));
            const uint32_t e_lo = from_row0(d_lo), e_hi = from_row0(d_hi);
            lo ^= ry ? e_lo : d_lo;
            hi ^= ry ? e_hi : d_hi;
            // rho (per-lane rotation) then pi (gather)
            const uint32_t a = swap ? hi : lo, b = swap ? lo : hi;
            const uint32_t na = __builtin_amdgcn_alignbit(a, b, sh), nb = __builtin_amdgcn_alignbit(b, a, sh);
            lo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(pisrc, static_cast<int>(na)));
            hi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(pisrc, static_cast<int>(nb)));
            // chi + iota (A(x + 1) / A(x + 2) inside the plane, wrapping by row shifts of 4 / 3)
            const uint32_t q_lo = sel(x4, dpp<kL4>(lo), dpp<kR1>(lo)), q_hi = sel(x4, dpp<kL4>(hi), dpp<kR1>(hi));
            const uint32_t r_lo = sel(x34, dpp<kL3>(lo), dpp<kR2>(lo)), r_hi = sel(x34, dpp<kL3>(hi), dpp<kR2>(hi));
            const uint64_t rc = kKeccakRC[round];
            lo = chi32(lo, q_lo, r_lo) ^ (static_cast<uint32_t>(rc) & m0);
            hi = chi32(hi, q_hi, r_hi) ^ (static_cast<uint32_t>(rc >> 32) & m0);
        }
    }
    // Keccak-256 of msg[0..len) (len a multiple of 8, msg 8-byte aligned, global or LDS memory);
    // lanes gl < 4 return digest word gl (bytes 8 gl .. 8 gl + 7) in lo/hi.
    __device__ __forceinline__ void hash(const uint8_t* msg, uint32_t len, uint32_t& lo, uint32_t& hi) const {
        lo = 0;
        hi = 0;
        const uint32_t nblocks = len / 136u + 1u;
        for (uint32_t blk = 0; blk < nblocks; ++blk) {
            const uint32_t pos = blk * 136u + 8u * static_cast<uint32_t>(gl);
            uint32_t wlo = 0, whi = 0;
            if (gl < 17) {
                if (pos < len) {
                    const uint2 w = *reinterpret_cast<const uint2*>(msg + pos);
                    wlo = w.x;
                    whi = w.y;
                } else if (pos == len) {
                    wlo = 1u;  // Keccak pad byte 0x01 (OpenSSLHasher.h:74-79)
                }
                if (blk + 1 == nblocks && gl == 16) whi ^= 0x80000000u;  // final 0x80
            }
            lo ^= wlo;
            hi ^= whi;
            permute(lo, hi);
        }
    }
};

// ------------------------------------------------------------------ lane-pair Keccak-256
// One state over two adjacent lanes (2k, 2k + 1): the even lane holds the low 32-bit halves of the 25
// 64-bit Keccak lanes, the odd lane the high halves.  theta's column parities, the theta XOR, chi and
// iota are lane-local; a 64-bit rotation of a (lo, hi) pair is, in BOTH lanes, one v_alignbit of the
// lane's own half and its partner's (rotl r < 32: alignbit(own, partner, 32 - r); r > 32:
// alignbit(partner, own, 64 - r)), the partner half fetched by one DPP quad_perm swap.  A round is
// ~120 VALU per lane (10 parity + 25 theta + 29 swaps + 29 alignbit + 25 chi + iota) against ~180 for a
// whole state in one lane, with no LDS and no cross-row traffic, so a latency-bound hash (a Merkle
// level with fewer nodes than the GPU has lanes) runs at two lanes per state.
struct KeccakPair {
    uint32_t odd;  // 0 on the even (low-half) lane, all-ones on the odd (high-half) lane
    __device__ KeccakPair() : odd(0u - (__lane_id() & 1u)) {}
    __device__ __forceinline__ static uint32_t partner(uint32_t v) {  // quad_perm [1, 0, 3, 2]
        return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xf, 0xf, false));
    }
    template <int R>
    __device__ __forceinline__ static uint32_t rot(uint32_t own, uint32_t par) {
        if constexpr (R == 0) return own;
        else if constexpr (R < 32) return __builtin_amdgcn_alignbit(own, par, 32 - R);
        else return __builtin_amdgcn_alignbit(par, own, 64 - R);
    }
    __device__ __forceinline__ void permute(uint32_t a[25]) const {
#pragma unroll 1
        for (int round = 0; round < 24; ++round) {
            const uint64_t rc64 = kKeccakRC[round];
            uint32_t c[5], e[5], t[25], b[25];
#pragma unroll
            for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(a[x], a[x + 5], a[x + 10]), a[x + 15], a[x + 20]);
#pragma unroll
            for (int x = 0; x < 5; ++x) {
                const uint32_t cx = c[(x + 1) % 5];
                e[x] = rot<1>(cx, partner(cx));
            }
#pragma unroll
            for (int i = 0; i < 25; ++i) t[i] = xor3(a[i], c[(i + 4) % 5], e[i % 5]);
            // rho + pi: b[y + 5((2x + 3y) % 5)] = rotl(t[x + 5y], r[x][y])
#define KP_RP(SRC, R, DST) b[DST] = rot<R>(t[SRC], R ? partner(t[SRC]) : 0u)
            KP_RP(0, 0, 0);   KP_RP(1, 1, 10);  KP_RP(2, 62, 20); KP_RP(3, 28, 5);  KP_RP(4, 27, 15);
            KP_RP(5, 36, 16); KP_RP(6, 44, 1);  KP_RP(7, 6, 11);  KP_RP(8, 55, 21); KP_RP(9, 20, 6);
            KP_RP(10, 3, 7);  KP_RP(11, 10, 17); KP_RP(12, 43, 2); KP_RP(13, 25, 12); KP_RP(14, 39, 22);
            KP_RP(15, 41, 23); KP_RP(16, 45, 8); KP_RP(17, 15, 18); KP_RP(18, 21, 3); KP_RP(19, 8, 13);
            KP_RP(20, 18, 14); KP_RP(21, 2, 24); KP_RP(22, 61, 9); KP_RP(23, 56, 19); KP_RP(24, 14, 4);
#undef KP_RP
#pragma unroll
            for (int y = 0; y < 25; y += 5) {
#pragma unroll
                for (int x = 0; x < 5; ++x) a[y + x] = chi32(b[y + x], b[y + (x + 1) % 5], b[y + (x + 2) % 5]);
            }
            const uint32_t rlo = static_cast<uint32_t>(rc64), rhi = static_cast<uint32_t>(rc64 >> 32);
            a[0] ^= (rlo & ~odd) | (rhi & odd);
        }
    }
    // Keccak-256 of msg[0..len) (len a multiple of 4, msg 4-byte aligned, global or LDS memory): the even lane absorbs the
    // low word of every 8-byte block lane, the odd lane the high word.  Returns digest words 2j + half
    // (half = this lane's) in d[j], j < 4.
    __device__ __forceinline__ void hash(const uint8_t* msg, uint32_t len, uint32_t d[4]) const {
        uint32_t a[25];
#pragma unroll
        for (int i = 0; i < 25; ++i) a[i] = 0;
        const uint32_t half = odd & 1u;
        const uint32_t nblocks = len / 136u + 1u;
        const uint32_t padw = len >> 2, padb = (len & 3u) * 8u;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(msg);
        const uint32_t nw = (len + 3u) >> 2;
        for (uint32_t blk = 0; blk < nblocks; ++blk) {
#pragma unroll
            for (int j = 0; j < 17; ++j) {
                const uint32_t wi = blk * 34u + 2u * j + half;
                uint32_t v = wi < nw ? w[wi] : 0u;
                if (wi == padw) v ^= 1u << padb;  // Keccak pad byte 0x01 (OpenSSLHasher.h:74-79)
                a[j] ^= v;
            }
            if (blk + 1 == nblocks) a[16] ^= 0x80000000u & odd;  // final 0x80
            permute(a);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = a[j];
    }
};

// Store a 32-byte digest.  Keccak words are little-endian lanes (byte order == memory order);
// SM3 words are big-endian.
__device__ __forceinline__ void store_digest(int hasher, uint8_t* dst, const uint32_t d[8]) {
    uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = hasher == SM3 ? bswap32(d[i]) : d[i];
}

}  // namespace bcosgpu
