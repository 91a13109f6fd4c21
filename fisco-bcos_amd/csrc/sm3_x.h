// sm3_x.h -- SM3 for Merkle nodes with the message expansion off the serial chain of compressions, and
// the constant padding block of a 64-byte (width-2) node.  Same digests as hash_device.h's sm3_msg
// (GB/T 32905-2016; SM3::hash, bcos-crypto/hasher/OpenSSLHasher.h:113-116); used by hash_kernels.hip.
#pragma once
#include "hash_device.h"

namespace bcosgpu {

// ------------------------------------------------------------------ SM3 with the expansion off the chain
// A block's message expansion depends only on the block, so for a multi-block message, or a level of
// many nodes, the expansions of all blocks can run at once (one lane per block) ahead of the serial
// compressions, which then read W[0..67] from LDS (kSm3Exp words, 16-byte aligned: b128 reads) and form
// W'[j] = W[j] ^ W[j + 4] themselves: a round loses the expansion's ~8 VALU ops (rounds 12..63) from the
// chain and gains one xor.
static constexpr uint32_t kSm3Exp = 68;

// block `blk` of the SM3 padding of the len-byte message m (len a multiple of 4, nw = len / 4 >= 1
// words, nblocks = (len + 8) / 64 + 1 blocks), as big-endian words -- sm3_msg's padding
__device__ __forceinline__ void sm3_load_block(const uint32_t* m, uint32_t len, uint32_t blk, uint32_t W[16]) {
    const uint32_t nw = len >> 2, nblocks = (len + 8u) / 64u + 1u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t idx = 16u * blk + k;
        const uint32_t v = m[idx < nw ? idx : nw - 1u];
        W[k] = (idx < nw ? bswap32(v) : 0u) ^ (idx == nw ? 0x80000000u : 0u);
    }
    if (blk + 1u == nblocks) {
        W[14] = 0u;  // bit length < 2^32
        W[15] = len * 8u;
    }
}

__device__ __forceinline__ void sm3_expand_block(const uint32_t W0[16], uint32_t* wx) {
    uint32_t W[68];
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = W0[j];
#pragma unroll
    for (int t = 16; t < 68; ++t)
        W[t] = xor3(sm3_p1(xor3(W[t - 16], W[t - 9], rotl32(W[t - 3], 15))), rotl32(W[t - 13], 7), W[t - 6]);
    uint4* o = reinterpret_cast<uint4*>(wx);
#pragma unroll
    for (int q = 0; q < 17; ++q) o[q] = make_uint4(W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]);
}

template <bool LOW>
__device__ __forceinline__ void sm3_round_x(int j, uint32_t wj, uint32_t wpj, uint32_t& A, uint32_t& B, uint32_t& C,
                                            uint32_t& D, uint32_t& E, uint32_t& F, uint32_t& G, uint32_t& H) {
    const uint32_t T = LOW ? 0x79cc4519u : 0x7a879d8au;
    const uint32_t a12 = rotl32(A, 12);
    const uint32_t SS1 = rotl32(a12 + E + rotl32(T, j & 31), 7);
    const uint32_t SS2 = SS1 ^ a12;
    const uint32_t FF = __builtin_amdgcn_bitop3_b32(A, B, C, LOW ? 0x96 : 0xE8);
    const uint32_t GG = __builtin_amdgcn_bitop3_b32(E, F, G, LOW ? 0x96 : 0xCA);
    const uint32_t TT1 = FF + D + SS2 + wpj;
    const uint32_t TT2 = GG + H + SS1 + wj;
    D = C; C = rotl32(B, 9); B = A; A = TT1;
    H = G; G = rotl32(F, 19); F = E; E = sm3_p0(TT2);
}

// The padding block of a 64-byte message (a width-2 Merkle node: 0x80, zeros, bit length 512) is a
// constant, so its expansion is a compile-time table and its compression takes W and W' as literals.
struct Sm3PadW {
    uint32_t w[68];
};
constexpr uint32_t sm3_rotl_c(uint32_t x, int r) { return r ? (x << r) | (x >> (32 - r)) : x; }
constexpr Sm3PadW sm3_pad64_w() {
    Sm3PadW p{};
    p.w[0] = 0x80000000u;
    p.w[15] = 512u;
    for (int t = 16; t < 68; ++t) {
        uint32_t x = p.w[t - 16] ^ p.w[t - 9] ^ sm3_rotl_c(p.w[t - 3], 15);
        x = x ^ sm3_rotl_c(x, 15) ^ sm3_rotl_c(x, 23);
        p.w[t] = x ^ sm3_rotl_c(p.w[t - 13], 7) ^ p.w[t - 6];
    }
    return p;
}
__device__ __forceinline__ void sm3_compress_pad64(uint32_t V[8]) {
    constexpr Sm3PadW P = sm3_pad64_w();
    uint32_t A = V[0], B = V[1], C = V[2], D = V[3], E = V[4], F = V[5], G = V[6], H = V[7];
#pragma unroll
    for (int j = 0; j < 16; ++j) sm3_round_x<true>(j, P.w[j], P.w[j] ^ P.w[j + 4], A, B, C, D, E, F, G, H);
#pragma unroll
    for (int j = 16; j < 64; ++j) sm3_round_x<false>(j, P.w[j], P.w[j] ^ P.w[j + 4], A, B, C, D, E, F, G, H);
    V[0] ^= A; V[1] ^= B; V[2] ^= C; V[3] ^= D; V[4] ^= E; V[5] ^= F; V[6] ^= G; V[7] ^= H;
}

// SM3 of a 64-byte message through a reader: one compression of its words, one of the constant padding
template <class Reader>
__device__ __forceinline__ void sm3_msg64(const Reader& rd, uint32_t out[8]) {
    uint32_t W[16];
    sm3_init(out);
#pragma unroll
    for (int j = 0; j < 16; ++j) W[j] = bswap32(rd.word(j));
    sm3_compress(out, W);
    sm3_compress_pad64(out);
}

// SM3 of a Merkle node (len = 32 x children bytes, 4-byte aligned): sm3_msg's digest, with every block
// that lies wholly inside the message read as four 16-byte loads (one lane reads one node: sixteen
// dword loads per block touched sixteen times as many cache lines per instruction)
__device__ __forceinline__ void sm3_node_msg(const uint8_t* src, uint32_t len, uint32_t out[8]) {
    sm3_init(out);
    const uint32_t nw = len >> 2, nblocks = (len + 8u) / 64u + 1u;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(src);
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        uint32_t W[16];
        const uint32_t w0 = blk * 16u;
        if (w0 + 16u <= nw && (reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
            const uint4* v = reinterpret_cast<const uint4*>(q + w0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 x = v[k];
                W[4 * k] = bswap32(x.x);
                W[4 * k + 1] = bswap32(x.y);
                W[4 * k + 2] = bswap32(x.z);
                W[4 * k + 3] = bswap32(x.w);
            }
        } else {
            sm3_load_block(q, len, blk, W);
        }
        sm3_compress(out, W);
    }
}

// one compression from an expanded block in LDS
__device__ __forceinline__ void sm3_compress_x(uint32_t V[8], const uint32_t* wx) {
    const uint4* w = reinterpret_cast<const uint4*>(wx);
    uint32_t A = V[0], B = V[1], C = V[2], D = V[3], E = V[4], F = V[5], G = V[6], H = V[7];
    uint4 a = w[0];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint4 n = w[q + 1];
        if (q < 4) {
            sm3_round_x<true>(4 * q, a.x, a.x ^ n.x, A, B, C, D, E, F, G, H);
            sm3_round_x<true>(4 * q + 1, a.y, a.y ^ n.y, A, B, C, D, E, F, G, H);
            sm3_round_x<true>(4 * q + 2, a.z, a.z ^ n.z, A, B, C, D, E, F, G, H);
            sm3_round_x<true>(4 * q + 3, a.w, a.w ^ n.w, A, B, C, D, E, F, G, H);
        } else {
            sm3_round_x<false>(4 * q, a.x, a.x ^ n.x, A, B, C, D, E, F, G, H);
            sm3_round_x<false>(4 * q + 1, a.y, a.y ^ n.y, A, B, C, D, E, F, G, H);
            sm3_round_x<false>(4 * q + 2, a.z, a.z ^ n.z, A, B, C, D, E, F, G, H);
            sm3_round_x<false>(4 * q + 3, a.w, a.w ^ n.w, A, B, C, D, E, F, G, H);
        }
        a = n;
    }
    V[0] ^= A; V[1] ^= B; V[2] ^= C; V[3] ^= D; V[4] ^= E; V[5] ^= F; V[6] ^= G; V[7] ^= H;
}

}  // namespace bcosgpu
