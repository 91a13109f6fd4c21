// hash_kernels.hip -- batch hashing and Merkle level kernels (gfx950).
//
// Replaces, for batches:
//   Hash::hash(bytesConstRef)             bcos-crypto/bcos-crypto/interfaces/crypto/Hash.h:44
//     (Keccak256::hash hash/Keccak256.h:39-51, SM3::hash hash/SM3.h:39-50)
//   Merkle<Hasher,width>::generateMerkle  bcos-crypto/bcos-crypto/merkle/Merkle.h:170-208
//     (per-level calculateLevelHashes :243-261 -> merkle_level_kernel, one node per lane)
//   protocol::calculateMerkleProofRoot    bcos-protocol/bcos-protocol/ParallelMerkleProof.cpp:32-69
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <mutex>
#include <utility>
#include <thread>
#include <vector>
#include "hash_device.h"
#include "sm3_x.h"
#include "engine.h"

namespace bcosgpu {

// One message per lane; message i = data[off[i] .. off[i+1]).
template <int H>
__global__ __launch_bounds__(256) void hash_batch_kernel(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ off,
                                                         uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = off[i], b = off[i + 1];
    const uint32_t len = static_cast<uint32_t>(b - a);
    FlatReader rd(data + a, len);
    uint32_t d[8];
    if (H == KECCAK256) keccak256_msg(rd, len, d);
    else sm3_msg(rd, len, d);
    store_digest(H, out + 32 * i, d);
}

// One Merkle node per lane: out[i] = H(in[i*W] || ... || in[min((i+1)*W, nin) - 1]).
// W = 0 selects the runtime width `w`.
template <int H, int W>
__global__ __launch_bounds__(256) void merkle_level_kernel(const uint8_t* __restrict__ in,
                                                           uint64_t nin, int w,
                                                           uint8_t* __restrict__ out,
                                                           uint64_t nout) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nout) return;
    const uint64_t width = W ? W : w;
    const uint64_t first = i * width;
    const uint64_t cnt = (nin - first) < width ? (nin - first) : width;
    const uint32_t len = static_cast<uint32_t>(cnt * 32u);
    NodeReader rd(in + first * 32, len);
    uint32_t d[8];
    if (H == KECCAK256) keccak256_msg(rd, len, d);
    else sm3_msg(rd, len, d);
    store_digest(H, out + 32 * i, d);
}

// Count records of the reference's output vector (Merkle.h:189-204, setNumberToHash :213-217):
// entry = uint32 big-endian level size in bytes 0..3, zero elsewhere.
struct LevelTable {
    uint64_t pos[64];
    uint32_t count[64];
    int nlevels;
};
__global__ void merkle_counts_kernel(uint8_t* tree, LevelTable t) {
    const int l = threadIdx.x;
    if (l >= t.nlevels) return;
    uint32_t* e = reinterpret_cast<uint32_t*>(tree + 32 * t.pos[l]);
    e[0] = bswap32(t.count[l]);
#pragma unroll
    for (int k = 1; k < 8; ++k) e[k] = 0;
}

// root = H(top) of the legacy algorithm (ParallelMerkleProof.cpp:68); len 0 -> H("") (:35-38).
template <int H>
__global__ void hash_one_kernel(const uint8_t* in, uint32_t len, uint8_t* out) {
    if (threadIdx.x != 0) return;
    AlignedReader rd(in, len);
    uint32_t d[8];
    if (H == KECCAK256) keccak256_msg(rd, len, d);
    else sm3_msg(rd, len, d);
    store_digest(H, out, d);
}

__global__ void copy32_kernel(const uint8_t* src, uint8_t* dst) {
    if (threadIdx.x < 8)
        reinterpret_cast<uint32_t*>(dst)[threadIdx.x] = reinterpret_cast<const uint32_t*>(src)[threadIdx.x];
}

static inline unsigned grid_for(uint64_t n, unsigned bs) { return static_cast<unsigned>((n + bs - 1) / bs); }

int launch_hash_batch(int hasher, const uint8_t* d_data, const uint64_t* d_off, uint64_t n,
                      uint8_t* d_out, hipStream_t st) {
    if (n == 0) return 0;
    if (hasher == SM3)
        hipLaunchKernelGGL(hash_batch_kernel<SM3>, dim3(grid_for(n, 256)), dim3(256), 0, st, d_data, d_off, n, d_out);
    else
        hipLaunchKernelGGL(hash_batch_kernel<KECCAK256>, dim3(grid_for(n, 256)), dim3(256), 0, st, d_data, d_off, n, d_out);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

static void launch_level(int hasher, int width, const uint8_t* in, uint64_t nin, uint8_t* out,
                         uint64_t nout, hipStream_t st) {
    dim3 g(grid_for(nout, 256)), b(256);
#define LVL(HH, WW) hipLaunchKernelGGL((merkle_level_kernel<HH, WW>), g, b, 0, st, in, nin, width, out, nout)
    if (hasher == SM3) {
        if (width == 2) LVL(SM3, 2); else if (width == 16) LVL(SM3, 16); else LVL(SM3, 0);
    } else {
        if (width == 2) LVL(KECCAK256, 2); else if (width == 16) LVL(KECCAK256, 16); else LVL(KECCAK256, 0);
    }
#undef LVL
}

uint64_t merkle_size(uint64_t n, int width) {
    uint64_t nodes = 0;
    while (n > 1) {
        n = (n + width - 1) / width;
        nodes += n + 1;
    }
    return nodes;
}

// ------------------------------------------------------------------ fused Merkle tree (2 launches)
// At merkleBench sizes the tree is latency-bound (a 512-byte width-16 node is 4 serial Keccak-f in one
// lane), so the per-level launches of the generic path cost as much as the hashing at the top.  Here
// one workgroup of B = width^k threads (the largest power of width <= 256) hashes B level-1 nodes and
// then every level whose groups lie inside it, through LDS, writing each node into the reference's
// output vector as it goes (groups align with workgroups because B is a power of width); a single
// 1024-thread workgroup then finishes the top levels.  Same output vector as the per-level path.
struct TreeLevels {
    uint64_t pos[64];  // tree entry of the count record of level l + 1 (level 0 = leaves)
    uint64_t cnt[64];  // nodes of level l + 1
    int nlev;          // levels above the leaves (the last has one node)
};

template <int H>
__device__ __forceinline__ void hash_nodes(const uint8_t* src, uint32_t cnt, uint32_t d[8]) {
    const uint32_t len = cnt * 32u;
    NodeReader rd(src, len);  // cnt >= 1
    if (H == KECCAK256) keccak256_msg(rd, len, d);
    else if (cnt == 2) sm3_msg64(rd, d);  // a full width-2 node: constant padding block
    else sm3_node_msg(src, len, d);
}

// SM3 of one node (c children: 32c bytes at buf, in LDS) by a whole wave: lanes 0 .. XB - 1 expand up
// to XB of its blocks at once into wx (XB * kSm3Exp words of LDS), then every lane runs the compressions
// from wx (uniform addresses: broadcast reads); the digest ends on every lane.
template <uint32_t XB>
__device__ __forceinline__ void sm3_node_lds(const uint8_t* buf, uint32_t c, uint32_t* wx, uint32_t d[8]) {
    const uint32_t lane = __lane_id();
    const uint32_t len = 32u * c, nblocks = (len + 8u) / 64u + 1u;
    sm3_init(d);
    for (uint32_t b0 = 0; b0 < nblocks; b0 += XB) {
        const uint32_t nb = nblocks - b0 < XB ? nblocks - b0 : XB;
        if (lane < nb) {
            uint32_t W[16];
            sm3_load_block(reinterpret_cast<const uint32_t*>(buf), len, b0 + lane, W);
            sm3_expand_block(W, wx + kSm3Exp * lane);
        }
        __syncthreads();
        for (uint32_t b = 0; b < nb; ++b) sm3_compress_x(d, wx + kSm3Exp * b);
        __syncthreads();  // before the next chunk's expansions overwrite wx
    }
}

// One SM3 level of nout nodes (their children at `in`, LDS or global, nin of them) with the message
// expansions of all its blocks at once -- thread t expands block t % nb of node t / nb into wx (nb = the
// blocks of a full node) -- then one thread per node runs its compressions from wx and writes the digest
// to dst + 32 j (and dst2 + 32 j when non-null).  The caller guarantees nout * nb <= blockDim.x and wx of
// that many blocks (sm3_level_fits), and a barrier between levels.
__device__ __forceinline__ uint32_t sm3_node_blocks(uint32_t width) { return (32u * width + 8u) / 64u + 1u; }
__device__ __forceinline__ bool sm3_level_fits(uint64_t nout, uint32_t width, uint32_t cap_blocks) {
    // (width 2: a full node's second block is the constant padding, which sm3_msg64 takes as literals)
    const uint32_t lim = blockDim.x < cap_blocks ? blockDim.x : cap_blocks;
    return width > 2 && nout * sm3_node_blocks(width) <= lim;
}
__device__ __forceinline__ void sm3_level_x(const uint8_t* in, uint64_t nin, uint32_t width, uint32_t nout, uint32_t* wx,
                                            uint8_t* dst, uint8_t* dst2) {
    const uint32_t tid = threadIdx.x;
    const uint32_t nb = sm3_node_blocks(width);
    {
        const uint32_t j = tid / nb, b = tid - j * nb;
        const uint64_t first = static_cast<uint64_t>(j) * width;
        const uint32_t c = j < nout ? static_cast<uint32_t>(nin - first < width ? nin - first : width) : 1u;
        if (j < nout && b < (32u * c + 8u) / 64u + 1u) {
            uint32_t W[16];
            sm3_load_block(reinterpret_cast<const uint32_t*>(in + 32ull * first), 32u * c, b, W);
            sm3_expand_block(W, wx + kSm3Exp * tid);
        }
    }
    __syncthreads();
    if (tid < nout) {
        const uint64_t first = static_cast<uint64_t>(tid) * width;
        const uint32_t c = static_cast<uint32_t>(nin - first < width ? nin - first : width);
        const uint32_t nblk = (32u * c + 8u) / 64u + 1u;
        uint32_t V[8];
        sm3_init(V);
        for (uint32_t b = 0; b < nblk; ++b) sm3_compress_x(V, wx + kSm3Exp * (tid * nb + b));
        store_digest(SM3, dst + 32ull * tid, V);
        if (dst2) store_digest(SM3, dst2 + 32ull * tid, V);
    }
}

// blocks of a width-W node's message (32W bytes + padding) expanded at once by sm3_node_lds
template <int W>
constexpr uint32_t sm3_node_xb() {
    return W && (32u * W + 8u) / 64u + 1u < 16u ? (32u * W + 8u) / 64u + 1u : 16u;
}

// One tree node cooperatively: every 32-lane group of the workgroup hashes node `base + group` of a
// level (Keccak only; all groups of a wave run the permutation together, idle ones on a dummy input).
// Lanes 0..3 of a group write the digest to dst (and dst2 when non-null).
template <int W>
__device__ __forceinline__ void coop_level_pass(const KeccakCoop& kc, const uint8_t* in, uint64_t nin, uint32_t width,
                                                uint64_t j, uint64_t nout, uint8_t* dst, uint8_t* dst2) {
    const bool act = j < nout;
    const uint64_t first = act ? j * width : 0;
    const uint32_t c = act ? static_cast<uint32_t>(nin - first < width ? nin - first : width) : 1u;
    uint32_t lo, hi;
    kc.hash(in + 32ull * first, 32u * c, lo, hi);
    if (act && kc.gl < 4) {
        *reinterpret_cast<uint2*>(dst + 8 * kc.gl) = make_uint2(lo, hi);
        if (dst2) *reinterpret_cast<uint2*>(dst2 + 8 * kc.gl) = make_uint2(lo, hi);
    }
}

// One tree node per lane PAIR (KeccakPair): lanes 2j, 2j + 1 hash node j of a level (idle pairs on a
// dummy input, so whole pairs stay in step); each lane writes its four digest words (2k + half) to
// dst + 32 j (and dst2 + 32 j when non-null).
__device__ __forceinline__ void pair_level_pass(const KeccakPair& kp, const uint8_t* in, uint64_t nin, uint32_t width,
                                                uint64_t j, uint64_t nout, uint8_t* dst, uint8_t* dst2) {
    const bool act = j < nout;
    const uint64_t first = act ? j * width : 0;
    const uint32_t c = act ? static_cast<uint32_t>(nin - first < width ? nin - first : width) : 1u;
    uint32_t d[4];
    kp.hash(in + 32ull * first, 32u * c, d);
    if (act) {
        const uint32_t half = __lane_id() & 1u;
        uint32_t* o = reinterpret_cast<uint32_t*>(dst + 32ull * j) + half;
        uint32_t* o2 = dst2 ? reinterpret_cast<uint32_t*>(dst2 + 32ull * j) + half : nullptr;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o[2 * k] = d[k];
            if (o2) o2[2 * k] = d[k];
        }
    }
}

// How a latency-bound Keccak level is hashed: 25 lanes per node while the level fits one node per
// 32-lane group, two lanes per node while it fits one node per lane pair (and `pair` allows it),
// else one lane per node.
enum LevelMode : int { kOneLane = 0, kPair = 1, kCoop = 2 };
template <int H>
__device__ __forceinline__ int level_mode(uint64_t nout, uint32_t threads, int pair, uint32_t coop_max = ~0u,
                                          uint32_t pair_max = ~0u) {
    if (H != KECCAK256) return kOneLane;
    if (nout <= threads / 32 && nout <= coop_max) return kCoop;
    if (pair && 2 * nout <= threads && nout <= pair_max) return kPair;
    return kOneLane;
}

// The workgroup's levels: its B level-1 nodes from the leaves, then every level whose groups lie inside
// it, through LDS (levels of at most coop_max nodes per full workgroup on 25-lane groups); returns the
// LDS buffer of the last level (whose first node is the workgroup's node `base` of that level).  Levels of
// more than pair_max nodes per full workgroup stay one lane per node.
// `pair`: level 1 (from the leaves) and the LDS levels may run on lane pairs (the host sets it when
// the tree's level 1 leaves most of the GPU idle; a throughput-sized level 1 stays one lane per node,
// which costs fewer instructions per node)
// X (SM3): levels whose blocks fit kWgXBlocks at once expand them in parallel (sm3_level_x, wx)
#ifdef BCOSGPU_MERKLE_PROBE  // tools/fusedprobe.hip, climbprobe.hip: per-wave / per-workgroup global timestamps (s_memrealtime, 100 MHz)
__device__ uint64_t g_mp[4096][40];
#define MP(k) \
    if (threadIdx.x == 0 && blockIdx.x < 4096 && (k) < 40) g_mp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime()
#else
#define MP(k) \
    do {      \
    } while (0)
#endif
static constexpr uint32_t kWgXBlocks = 256, kTopXBlocks = 448;
template <int H, int W, bool X = false>
__device__ __forceinline__ int wg_levels(uint4 (*lds)[256][2], const uint8_t* __restrict__ leaves, uint64_t n,
                                         uint32_t width, int kin, int B, uint8_t* __restrict__ tree, const TreeLevels& t,
                                         int pair, uint32_t coop_max, uint32_t pair_max, uint64_t& base,
                                         uint32_t* wx = nullptr) {
    const uint32_t tid = threadIdx.x;
    base = static_cast<uint64_t>(blockIdx.x) * B;  // first level-1 node of this workgroup
    uint32_t nodes = static_cast<uint32_t>(t.cnt[0] - base < static_cast<uint64_t>(B) ? t.cnt[0] - base : B);
    uint32_t d[8];
    if (level_mode<H>(B, blockDim.x, pair, ~0u, pair_max) == kPair) {
        const KeccakPair kp;
        pair_level_pass(kp, leaves + 32ull * base * width, n - base * width, width, tid >> 1, nodes,
                        tree + 32ull * (t.pos[0] + 1 + base), reinterpret_cast<uint8_t*>(&lds[0][0][0]));
    } else if (tid < nodes) {
        const uint64_t first = (base + tid) * width;
        const uint32_t c = static_cast<uint32_t>(n - first < width ? n - first : width);
        hash_nodes<H>(leaves + 32ull * first, c, d);
        store_digest(H, tree + 32ull * (t.pos[0] + 1 + base + tid), d);
        store_digest(H, reinterpret_cast<uint8_t*>(&lds[0][tid][0]), d);
    }
    int cur = 0;
    MP(20);
    const int top = kin + 1 < t.nlev ? kin + 1 : t.nlev;  // levels this kernel produces
    for (int l = 1; l < top; ++l) {
        __syncthreads();
        const uint64_t nbase = base / width;
        const uint32_t nn = (nodes + width - 1) / width;
        const uint8_t* in = reinterpret_cast<const uint8_t*>(&lds[cur][0][0]);
        // (the mode is decided on the full group count B / width^l so every workgroup runs alike)
        const int mode = level_mode<H>((B + width - 1) / width, blockDim.x, pair, coop_max, pair_max);
        if (mode == kCoop) {  // latency-bound level: 25 lanes per node
            const KeccakCoop kc;
            const uint32_t g = tid / 32;
            coop_level_pass<W>(kc, in, nodes, width, g, nn, tree + 32ull * (t.pos[l] + 1 + nbase + g),
                               reinterpret_cast<uint8_t*>(&lds[cur ^ 1][g < 256 ? g : 0][0]));
        } else if (mode == kPair) {
            const KeccakPair kp;
            pair_level_pass(kp, in, nodes, width, tid >> 1, nn, tree + 32ull * (t.pos[l] + 1 + nbase),
                            reinterpret_cast<uint8_t*>(&lds[cur ^ 1][0][0]));
        } else if (X && H == SM3 && sm3_level_fits(nn, width, kWgXBlocks)) {
            sm3_level_x(in, nodes, width, nn, wx, tree + 32ull * (t.pos[l] + 1 + nbase),
                        reinterpret_cast<uint8_t*>(&lds[cur ^ 1][0][0]));
        } else if (tid < nn) {
            const uint32_t c = nodes - tid * width < width ? nodes - tid * width : width;
            hash_nodes<H>(in + 32u * tid * width, c, d);
            store_digest(H, tree + 32ull * (t.pos[l] + 1 + nbase + tid), d);
            store_digest(H, reinterpret_cast<uint8_t*>(&lds[cur ^ 1][tid][0]), d);
        }
        cur ^= 1;
        nodes = nn;
        base = nbase;
        B = (B + width - 1) / width;
        MP(20 + l);
    }
    return cur;
}

template <int H, int W, bool X>
__global__ __launch_bounds__(512) void merkle_wg_kernel(const uint8_t* __restrict__ leaves, uint64_t n, int w, int kin,
                                                        int B, uint8_t* __restrict__ tree, const TreeLevels t,
                                                        uint8_t* __restrict__ root, int pair) {
    __shared__ uint4 lds[2][256][2];
    __shared__ uint4 wxs[X ? kWgXBlocks * kSm3Exp / 4 : 1];
    const uint32_t tid = threadIdx.x;
    uint64_t base;
    const int cur = wg_levels<H, W, X>(lds, leaves, n, W ? W : static_cast<uint32_t>(w), kin, B, tree, t, pair, ~0u,
                                       ~0u, base, reinterpret_cast<uint32_t*>(&wxs[0]));
    const int top = kin + 1 < t.nlev ? kin + 1 : t.nlev;
    if (blockIdx.x == 0 && tid < static_cast<uint32_t>(t.nlev)) {  // count records (Merkle.h:189-204)
        uint32_t* e = reinterpret_cast<uint32_t*>(tree + 32ull * t.pos[tid]);
        e[0] = bswap32(static_cast<uint32_t>(t.cnt[tid]));
#pragma unroll
        for (int k = 1; k < 8; ++k) e[k] = 0;
    }
    if (top == t.nlev && root) {  // the whole tree fit in this (single) workgroup
        __syncthreads();
        if (tid == 0) {
            const uint4* r = &lds[cur][0][0];
            reinterpret_cast<uint4*>(root)[0] = r[0];
            reinterpret_cast<uint4*>(root)[1] = r[1];
        }
    }
}

// levels [l0, t.nlev) (0-based, level l0 - 1 already in the tree) in ONE workgroup; root copy
template <int H, int W, bool X>
__global__ __launch_bounds__(1024) void merkle_top_kernel(int w, int l0, uint8_t* __restrict__ tree, const TreeLevels t,
                                                          uint8_t* __restrict__ root, int pair) {
    __shared__ uint4 wxs[X ? kTopXBlocks * kSm3Exp / 4 : 1];
    const uint32_t width = W ? W : static_cast<uint32_t>(w);
    for (int l = l0; l < t.nlev; ++l) {
        const uint64_t nin = t.cnt[l - 1];
        const uint8_t* in = tree + 32ull * (t.pos[l - 1] + 1);
        const int mode = level_mode<H>(t.cnt[l], blockDim.x, pair);
        if (X && H == SM3 && sm3_level_fits(t.cnt[l], width, kTopXBlocks)) {
            sm3_level_x(in, nin, width, static_cast<uint32_t>(t.cnt[l]), reinterpret_cast<uint32_t*>(&wxs[0]),
                        tree + 32ull * (t.pos[l] + 1), nullptr);
        } else if (mode == kCoop) {  // latency-bound level: 25 lanes per node
            const KeccakCoop kc;
            const uint32_t g = threadIdx.x / 32;
            coop_level_pass<W>(kc, in, nin, width, g, t.cnt[l], tree + 32ull * (t.pos[l] + 1 + g), nullptr);
        } else if (mode == kPair) {
            const KeccakPair kp;
            pair_level_pass(kp, in, nin, width, threadIdx.x >> 1, t.cnt[l], tree + 32ull * (t.pos[l] + 1), nullptr);
        } else {
            for (uint64_t j = threadIdx.x; j < t.cnt[l]; j += blockDim.x) {
                const uint64_t first = j * width;
                const uint32_t c = static_cast<uint32_t>(nin - first < width ? nin - first : width);
                uint32_t d[8];
                hash_nodes<H>(in + 32ull * first, c, d);
                store_digest(H, tree + 32ull * (t.pos[l] + 1 + j), d);
            }
        }
        __syncthreads();
    }
    if (root && threadIdx.x < 2) {
        const uint4* r = reinterpret_cast<const uint4*>(tree + 32ull * (t.pos[t.nlev - 1] + 1));
        reinterpret_cast<uint4*>(root)[threadIdx.x] = r[threadIdx.x];
    }
}

// ------------------------------------------------------------------ latency-sized trees: one launch
// At merkleBench sizes (100k leaves, width 16: 6,250 level-1 nodes) the tree is a chain of serial
// permutations, and what costs is how many of them share a SIMD: the workgroup-per-256-nodes kernel
// puts level 1 on 25 CUs at two waves per SIMD and the single-workgroup top kernel runs level 3's
// 25 cooperative hashes at four waves per SIMD.  Here every wave is its own workgroup (one wave per
// SIMD across the GPU): wave b hashes the S = width^a level-1 nodes under one level-(a+1) node (lane
// pairs for Keccak, one lane per node for SM3), the levels above them inside the wave through LDS
// (Keccak: pairs, then 25-lane groups for the last one or two nodes), and then climbs: it publishes
// its node and bumps the arrival counter of the parent, and the wave that completes a parent's group
// hashes the parent (one 25-lane group / one lane) and climbs on, up to the root.
// Cross-wave hand-off without cache-wide fences: a published node is written with device-coherent
// stores (agent-scope atomic stores: write-through past the per-XCD L2), the wave waits for them
// (s_waitcnt) before its counter atomic, and the completing wave gathers the children with
// device-coherent loads into LDS; the last arriver resets the counter, so the slot is clean for the
// next launch on the stream.  The ordering this rests on is the ISA's, not the language's (relaxed
// atomics order nothing between locations): agent-scope relaxed stores / loads are sc1 accesses,
// coherent at agent scope; "s_waitcnt vmcnt(0)" returns only once the stores are acknowledged; the
// counter RMW's return is waited for before the branch that leads to the loads; and compiler barriers
// ("memory" clobbers) keep the compiler from reordering across either point.  tests/test_hazards.py
// checks the emitted order on every build (tools/hazard_check.py fused_publish_order).  An acq_rel
// counter (the language-level form) costs a buffer_wbl2 / buffer_inv of the XCD's L2 per hand-off:
// 0.175 vs 0.130 ms per 100k-leaf width-2 Keccak root (profiles/r04_merkle_fused_order_ab.log).
struct FusedTree {
    TreeLevels t;
    uint32_t ctr_off[64];  // first counter of level l (levels a + 1 .. nlev - 1)
    int a;                 // levels above level 1 computed inside a wave (S = width^a)
    uint32_t S;
};

__device__ __forceinline__ void st_dev(uint8_t* p, uint32_t v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_dev(const uint8_t* p) {
    return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// hash node j of a level from its children at `in` (nin of them) -- gathered into LDS `buf` with
// device-coherent loads -- with one 25-lane group (Keccak; group 1 hashes a dummy copy) or the whole
// wave (SM3, sm3_node_lds over wx); publishes the digest at dst with device-coherent stores
template <int H, int W>
__device__ __forceinline__ void fused_one_node(const uint8_t* in, uint64_t nin, uint32_t width, uint64_t j,
                                               uint8_t* dst, uint8_t* buf, uint32_t* wx) {
    const uint64_t first = j * width;
    const uint32_t c = static_cast<uint32_t>(nin - first < width ? nin - first : width);
    const uint32_t lane = __lane_id();
    for (uint32_t q = lane; q < 8u * c; q += 64u)
        reinterpret_cast<uint32_t*>(buf)[q] = ld_dev(in + 32ull * first + 4u * q);
    __syncthreads();
    if constexpr (H == KECCAK256) {
        const KeccakCoop kc;
        uint32_t lo, hi;
        kc.hash(buf, 32u * c, lo, hi);
        if (lane < 32 && kc.gl < 4) {
            st_dev(dst + 8 * kc.gl, lo);
            st_dev(dst + 8 * kc.gl + 4, hi);
        }
    } else {
        uint32_t d[8];
        sm3_node_lds<sm3_node_xb<W>()>(buf, c, wx, d);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) st_dev(dst + 4 * k, bswap32(d[k]));
        }
    }
}

// one level of a wave's subtree: `nodes` nodes (of `full` under a full wave) from `nin` children at
// `in`, written to the tree at dst (node k at dst + 32 k) and to LDS dl
template <int H, int W>
__device__ __forceinline__ void fused_level(const uint8_t* in, uint64_t nin, uint32_t width, uint32_t full,
                                            uint32_t nodes, uint8_t* dst, uint8_t* dl) {
    const uint32_t lane = __lane_id();
    if (H == KECCAK256 && full > 2) {  // lane pairs (uniform per level: decided on the full count)
        const KeccakPair kp;
        pair_level_pass(kp, in, nin, width, lane >> 1, nodes, dst, dl);
    } else if (H == KECCAK256) {      // one or two nodes: a 25-lane group each
        const KeccakCoop kc;
        coop_level_pass<W>(kc, in, nin, width, lane >> 5, nodes, dst + 32 * (lane >> 5), dl + 32 * (lane >> 5));
    } else if (lane < nodes) {
        uint32_t d[8];
        const uint64_t first = static_cast<uint64_t>(lane) * width;
        const uint32_t c = static_cast<uint32_t>(nin - first < width ? nin - first : width);
        hash_nodes<H>(in + 32ull * first, c, d);
        store_digest(H, dst + 32ull * lane, d);
        store_digest(H, dl + 32ull * lane, d);
    }
}


template <int H, int W>
__global__ __launch_bounds__(64) void merkle_fused_kernel(const uint8_t* __restrict__ leaves, uint64_t n, int w,
                                                          uint8_t* __restrict__ tree, const FusedTree f,
                                                          uint8_t* __restrict__ root, uint32_t* __restrict__ ctr) {
    __shared__ uint4 lds[2][64][2];
    __shared__ uint4 wxs[H == SM3 ? sm3_node_xb<W>() * kSm3Exp / 4 : 1];  // SM3 climb nodes' expanded blocks
    const TreeLevels& t = f.t;
    const uint32_t width = W ? W : static_cast<uint32_t>(w);
    const uint32_t lane = threadIdx.x;
    if (blockIdx.x == 0 && lane < static_cast<uint32_t>(t.nlev)) {  // count records (Merkle.h:189-204)
        uint32_t* e = reinterpret_cast<uint32_t*>(tree + 32ull * t.pos[lane]);
        e[0] = bswap32(static_cast<uint32_t>(t.cnt[lane]));
#pragma unroll
        for (int k = 1; k < 8; ++k) e[k] = 0;
    }
    // ---- level 0 (from the leaves, global memory) and levels 1 .. a inside the wave (from LDS); the
    // two kinds of source stay separate so every load has a known address space (no flat loads)
    MP(0);
    uint64_t base = static_cast<uint64_t>(blockIdx.x) * f.S;  // first level-0 node of this wave
    uint32_t nodes = static_cast<uint32_t>(t.cnt[0] - base < f.S ? t.cnt[0] - base : f.S);
    const int inner = f.a + 1 < t.nlev ? f.a + 1 : t.nlev;  // levels this wave computes before climbing
    fused_level<H, W>(leaves + 32ull * base * width, n - base * width, width, f.S, nodes,
                      tree + 32ull * (t.pos[0] + 1 + base), reinterpret_cast<uint8_t*>(&lds[0][0][0]));
    __syncthreads();
    MP(1);
    int cur = 0;
    uint32_t full = f.S;  // nodes of the level under a full wave
    for (int l = 1; l < inner; ++l) {
        const uint32_t nin = nodes;
        nodes = (nodes + width - 1) / width;
        base /= width;
        full /= width;
        fused_level<H, W>(reinterpret_cast<const uint8_t*>(&lds[cur][0][0]), nin, width, full, nodes,
                          tree + 32ull * (t.pos[l] + 1 + base), reinterpret_cast<uint8_t*>(&lds[cur ^ 1][0][0]));
        cur ^= 1;
        __syncthreads();
    }
    MP(2);
    // ---- climb: the wave completing a parent's group of children hashes the parent
    uint64_t j = base;  // this wave's node at level inner - 1 (lds[cur][0])
    if (inner < t.nlev && lane < 8)  // publish it (device-coherent)
        st_dev(tree + 32ull * (t.pos[inner - 1] + 1 + j) + 4 * lane, reinterpret_cast<const uint32_t*>(&lds[cur][0][0])[lane]);
    for (int l = inner; l < t.nlev; ++l) {
        const uint64_t p = j / width;
        const uint32_t kids = static_cast<uint32_t>(t.cnt[l - 1] - p * width < width ? t.cnt[l - 1] - p * width : width);
        uint32_t arrived = 0;
        // the published node's stores have completed (whole wave); the "memory" clobber also keeps the
        // compiler from moving any memory access across this point (relaxed atomics alone would allow it)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lane == 0) {
            uint32_t* c = ctr + f.ctr_off[l] + p;
            arrived = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            if (arrived == kids) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        arrived = __shfl(arrived, 0);
        if (arrived != kids) return;  // a sibling's wave finishes the parent
        asm volatile("" ::: "memory");  // the children's loads stay after the counter (compiler order)
        MP(3 + 2 * (l - inner));
        fused_one_node<H, W>(tree + 32ull * (t.pos[l - 1] + 1), t.cnt[l - 1], width, p, tree + 32ull * (t.pos[l] + 1 + p),
                             reinterpret_cast<uint8_t*>(&lds[0][0][0]), reinterpret_cast<uint32_t*>(&wxs[0]));
        MP(4 + 2 * (l - inner));
        j = p;
    }
    if (root && lane < 8 && j == 0) {  // this wave wrote the root node (or the whole tree fit in it)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        reinterpret_cast<uint32_t*>(root)[lane] = ld_dev(tree + 32ull * (t.pos[t.nlev - 1] + 1) + 4 * lane);
    }
}

// One counter slot (kFusedCounters counters) per launch queue: launches on one stream run in order and
// each launch leaves its counters at zero, so a slot is clean for the next launch of its owner.
//  - Owners: a created stream by its handle (hipStreamDestroy releases the stream object only once its
//    work has completed, so a handle that comes back for a new stream has no launch of the old one in
//    flight); the legacy null stream by its device (one in-order queue for every thread); the
//    per-thread default stream (hipStreamPerThread) by the calling thread, whose slot goes back to the
//    pool when that thread exits (after its stream drains).
//  - A new slot is zeroed by hipMemsetAsync on the claiming stream (ordered before its first launch; no
//    device-wide synchronisation), and a stream under capture never claims one (a capture may not
//    allocate): it takes the multi-launch path.
//  - Pools of kFusedSlots slots are added on demand up to kFusedPools per device; past that the
//    multi-launch path runs (bit-identical, slower at latency sizes) and a line on stderr says so once.
static constexpr uint32_t kFusedCounters = 16384, kFusedSlots = 64, kFusedPools = 16;
namespace {
struct SlotOwner {
    int device;
    int kind;  // 0 created stream (id), 1 legacy null stream, 2 per-thread default stream (thread), -1 free
    unsigned long long id;
    std::thread::id thread;
};
struct SlotPool {
    int device;
    uint32_t* base;
    std::vector<SlotOwner> owners;
};
std::mutex g_slot_mu;
std::vector<SlotPool>& slot_pools() {
    static std::vector<SlotPool>* pools = new std::vector<SlotPool>();  // never destroyed (exit order)
    return *pools;
}
// the calling thread's per-thread-stream slots, returned to their pools when the thread exits
struct PerThreadSlots {
    std::vector<std::pair<size_t, size_t>> held;  // (pool, slot)
    ~PerThreadSlots() {
        if (held.empty()) return;
        // drain this thread's per-thread stream on EVERY device it held a slot on (its last launches there
        // have reset their counters) before the slots go back: a slot is reused without a memset
        std::vector<int> devs;
        {
            std::lock_guard<std::mutex> g(g_slot_mu);
            for (auto& h : held) devs.push_back(slot_pools()[h.first].device);
        }
        int prev = -1;
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        std::vector<int> done;
        for (int d : devs) {
            if (std::find(done.begin(), done.end(), d) != done.end()) continue;
            done.push_back(d);
            if (hipSetDevice(d) == hipSuccess) (void)hipStreamSynchronize(hipStreamPerThread);
        }
        if (prev >= 0) (void)hipSetDevice(prev);
        (void)hipGetLastError();
        std::lock_guard<std::mutex> g(g_slot_mu);
        for (auto& h : held) slot_pools()[h.first].owners[h.second].kind = -1;
    }
};
thread_local PerThreadSlots t_slots;
}  // namespace

static uint32_t* fused_counter_slot(hipStream_t st) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    SlotOwner me{dev, 0, 0, std::thread::id()};
    if (st == nullptr) {
        me.kind = 1;
    } else if (st == hipStreamPerThread) {
        me.kind = 2;
        me.thread = std::this_thread::get_id();
    } else {
        hipDevice_t sd = 0;
        if (hipStreamGetDevice(st, &sd) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        me.id = static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(st));
        me.device = dev = sd;
    }
    std::lock_guard<std::mutex> g(g_slot_mu);
    std::vector<SlotPool>& pools = slot_pools();
    for (auto& q : pools) {
        if (q.device != dev) continue;
        for (size_t k = 0; k < q.owners.size(); ++k) {
            const SlotOwner& o = q.owners[k];
            if (o.kind == me.kind && o.id == me.id && o.thread == me.thread) return q.base + k * kFusedCounters;
        }
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (cap != hipStreamCaptureStatusNone) return nullptr;
    // a returned slot (zero counters: its thread's stream drained), else a new one in a pool with room
    size_t pi = pools.size(), si = 0;
    int npools = 0;
    for (size_t q = 0; q < pools.size() && pi == pools.size(); ++q) {
        if (pools[q].device != dev) continue;
        ++npools;
        for (size_t k = 0; k < pools[q].owners.size(); ++k)
            if (pools[q].owners[k].kind == -1) {
                pi = q;
                si = k;
                break;
            }
    }
    if (pi == pools.size()) {
        for (size_t q = 0; q < pools.size(); ++q)
            if (pools[q].device == dev && pools[q].owners.size() < kFusedSlots) {
                pi = q;
                si = pools[q].owners.size();
                break;
            }
    }
    if (pi == pools.size()) {
        if (npools >= static_cast<int>(kFusedPools)) {
            static std::atomic<bool> warned{false};
            if (!warned.exchange(true))
                std::fprintf(stderr, "bcosgpu: the one-launch Merkle path's %u counter slots on device %d are all "
                                     "owned (one per stream); further streams take the multi-launch path\n",
                             kFusedSlots * kFusedPools, dev);
            return nullptr;
        }
        int prev = dev;
        (void)hipGetDevice(&prev);
        if (prev != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
        void* b = nullptr;
        const hipError_t e = hipMalloc(&b, sizeof(uint32_t) * kFusedCounters * kFusedSlots);
        if (prev != dev) (void)hipSetDevice(prev);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        pools.push_back(SlotPool{dev, static_cast<uint32_t*>(b), {}});
        pi = pools.size() - 1;
        si = 0;
    }
    SlotPool& pool = pools[pi];
    uint32_t* slot = pool.base + si * kFusedCounters;
    const bool fresh = si == pool.owners.size();
    if (fresh && hipMemsetAsync(slot, 0, sizeof(uint32_t) * kFusedCounters, st) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (fresh)
        pool.owners.push_back(me);
    else
        pool.owners[si] = me;
    if (me.kind == 2) t_slots.held.emplace_back(pi, si);
    return slot;
}

static constexpr uint64_t kFusedMaxWaves = 2048;  // level-1 waves (two per SIMD) up to which the one-launch path runs

// the latency path; returns 1 when it does not apply (too wide a tree, no counter slot)
static int launch_merkle_fused(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                               uint8_t* d_root, const TreeLevels& t, bool force, hipStream_t st) {
    FusedTree f{};
    f.t = t;
    // S = width^a: Keccak level 0 on lane pairs (S <= 32), SM3 one lane per node (S <= 64)
    const uint32_t cap = hasher == KECCAK256 ? 32u : 64u;
    f.S = 1;
    f.a = 0;
    while (f.S * static_cast<uint32_t>(width) <= cap) {
        f.S *= width;
        ++f.a;
    }
    uint32_t off = 0;
    for (int l = 0; l < t.nlev; ++l) {
        f.ctr_off[l] = off;
        if (l > f.a) off += static_cast<uint32_t>(t.cnt[l]);
    }
    if (off > kFusedCounters || (!force && (t.cnt[0] + f.S - 1) / f.S > kFusedMaxWaves)) return 1;
    uint32_t* ctr = fused_counter_slot(st);
    if (!ctr) return 1;
    const dim3 g(static_cast<unsigned>((t.cnt[0] + f.S - 1) / f.S)), b(64);
#define FUSED(HH, WW) hipLaunchKernelGGL((merkle_fused_kernel<HH, WW>), g, b, 0, st, d_leaves, n, width, d_tree, f, d_root, ctr)
    if (hasher == SM3) {
        if (width == 2) FUSED(SM3, 2); else if (width == 16) FUSED(SM3, 16); else FUSED(SM3, 0);
    } else {
        if (width == 2) FUSED(KECCAK256, 2); else if (width == 16) FUSED(KECCAK256, 16); else FUSED(KECCAK256, 0);
    }
#undef FUSED
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

// ------------------------------------------------------------------ one launch, four-wave workgroups
// The one-launch path for narrow Keccak trees (the production width 2, Merkle.h:36 / BlockImpl.h:125).
// With one wave per workgroup (above) a width-2 tree needs 32 level-1 nodes per wave on lane pairs, i.e.
// 1,563 waves for 100k leaves -- two waves on many SIMDs -- and then five more lane-pair or 25-lane levels
// and a cross-wave hand-off for each of the 11 levels above.  Here a workgroup is four waves, one per SIMD
// of a CU: it hashes B = width^kin <= 256 level-1 nodes one lane each, the levels above them through LDS
// as merkle_wg_kernel does (lane pairs while a level has more than coop_max nodes, then 25-lane groups,
// eight per workgroup), and then climbs like merkle_fused_kernel, except that a climb step takes g levels
// at once: the workgroup completing a group of width^g nodes gathers them and hashes the g levels above
// with its eight 25-lane groups (width 2: 16 nodes -> 8 -> 4 -> 2 -> 1, one hand-off per four levels).
// The hand-off is merkle_fused_kernel's: sc1 node stores, s_waitcnt vmcnt(0) + barrier before the counter
// RMW, sc1 loads after it, compiler barriers at both points (tools/hazard_check.py checks the order).
struct ClimbTree {
    TreeLevels t;
    uint32_t ctr_off[64];  // first arrival counter of level l (the top level of a climb step)
    int kin;               // levels above level 1 inside a workgroup (B = width^kin)
    int B;
    int g;                 // levels per climb step: width^(g - 1) <= 8 first-level nodes (SM3: <= 64)
    uint32_t coop_max;     // in-workgroup levels of at most this many nodes run on 25-lane groups
    uint32_t pair_max;     // ... of at most this many (and more than coop_max) on lane pairs, else one lane
    int pair;
};

// X (SM3, latency-sized trees of width > 2): the in-workgroup levels above level 1 and the climb steps'
// levels expand their blocks in parallel first (sm3_level_x, as merkle_wg_kernel's X variant), so C1's SM3
// root (width 16) runs as ONE launch -- the last workgroup to finish its level-3 node climbs to the root --
// instead of merkle_wg_kernel + merkle_top_kernel
template <int H, int W, bool X = false>
__global__ __launch_bounds__(256) void merkle_climb_kernel(const uint8_t* __restrict__ leaves, uint64_t n, int w,
                                                           uint8_t* __restrict__ tree, const ClimbTree f,
                                                           uint8_t* __restrict__ root, uint32_t* __restrict__ ctr) {
    __shared__ uint4 lds[2][256][2];
    __shared__ uint4 wxs[X ? kWgXBlocks * kSm3Exp / 4 : 1];
    __shared__ uint32_t arrived_s;
    const TreeLevels& t = f.t;
    const uint32_t width = W ? W : static_cast<uint32_t>(w);
    const uint32_t tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < static_cast<uint32_t>(t.nlev)) {  // count records (Merkle.h:189-204)
        uint32_t* e = reinterpret_cast<uint32_t*>(tree + 32ull * t.pos[tid]);
        e[0] = bswap32(static_cast<uint32_t>(t.cnt[tid]));
#pragma unroll
        for (int k = 1; k < 8; ++k) e[k] = 0;
    }
    uint64_t j;  // this workgroup's node at level l - 1 (LDS buffer cur, entry 0)
    MP(0);
    int cur = wg_levels<H, W, X>(lds, leaves, n, width, f.kin, f.B, tree, t, f.pair, f.coop_max, f.pair_max, j,
                                 reinterpret_cast<uint32_t*>(&wxs[0]));
    MP(1);
    [[maybe_unused]] int step = 0;  // climb steps taken (the probe build's stamps)
    int l = f.kin + 1 < t.nlev ? f.kin + 1 : t.nlev;  // next level to compute
    __syncthreads();
    if (l < t.nlev && tid < 8)  // publish it (device-coherent)
        st_dev(tree + 32ull * (t.pos[l - 1] + 1 + j) + 4 * tid, reinterpret_cast<const uint32_t*>(&lds[cur][0][0])[tid]);
    while (l < t.nlev) {
        const int g = f.g < t.nlev - l ? f.g : t.nlev - l;
        uint64_t G = 1;
        for (int q = 0; q < g; ++q) G *= width;
        const uint64_t P = j / G, first = P * G;  // the step's top node (level l + g - 1), its first child
        const uint32_t kids = static_cast<uint32_t>(t.cnt[l - 1] - first < G ? t.cnt[l - 1] - first : G);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the published node's stores are acknowledged
        __syncthreads();
        if (tid == 0) {
            uint32_t* c = ctr + f.ctr_off[l + g - 1] + P;
            const uint32_t a = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            if (a == kids) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            arrived_s = a;
        }
        __syncthreads();
        if (arrived_s != kids) return;  // a sibling's workgroup climbs on
        asm volatile("" ::: "memory");  // the children's loads stay after the counter (compiler order)
        MP(2 + 2 * step);
        uint32_t* buf = reinterpret_cast<uint32_t*>(&lds[0][0][0]);
        const uint8_t* src = tree + 32ull * (t.pos[l - 1] + 1 + first);
        for (uint32_t q = tid; q < 8u * kids; q += 256u) buf[q] = ld_dev(src + 4u * q);
        __syncthreads();
        cur = 0;
        uint32_t nin = kids;
        uint64_t b = first;
        for (int i = 0; i < g; ++i) {
            const uint32_t nn = (nin + width - 1) / width;
            b /= width;
            const uint8_t* in = reinterpret_cast<const uint8_t*>(&lds[cur][0][0]);
            if constexpr (H == KECCAK256) {  // nn <= 8 nodes per level: one pass of the eight 32-lane groups
                const KeccakCoop kc;
                const uint32_t gq = tid / 32;
                coop_level_pass<W>(kc, in, nin, width, gq, nn, tree + 32ull * (t.pos[l + i] + 1 + b + gq),
                                   reinterpret_cast<uint8_t*>(&lds[cur ^ 1][gq < 8 ? gq : 0][0]));
            } else if (X && sm3_level_fits(nn, width, kWgXBlocks)) {  // SM3, blocks expanded at once
                sm3_level_x(in, nin, width, nn, reinterpret_cast<uint32_t*>(&wxs[0]),
                            tree + 32ull * (t.pos[l + i] + 1 + b), reinterpret_cast<uint8_t*>(&lds[cur ^ 1][0][0]));
            } else if (tid < nn) {  // SM3: one lane per node (nn <= 64)
                uint32_t d[8];
                const uint32_t c = nin - tid * width < width ? nin - tid * width : width;
                hash_nodes<H>(in + 32u * tid * width, c, d);
                store_digest(H, tree + 32ull * (t.pos[l + i] + 1 + b + tid), d);
                store_digest(H, reinterpret_cast<uint8_t*>(&lds[cur ^ 1][tid][0]), d);
            }
            cur ^= 1;
            nin = nn;
            __syncthreads();
        }
        j = P;
        l += g;
        MP(3 + 2 * step);
        ++step;
        if (l < t.nlev && tid < 8)
            st_dev(tree + 32ull * (t.pos[l - 1] + 1 + j) + 4 * tid, reinterpret_cast<const uint32_t*>(&lds[cur][0][0])[tid]);
    }
    if (root && j == 0 && tid < 8)  // this workgroup produced the root node (or the whole tree fit in it)
        reinterpret_cast<uint32_t*>(root)[tid] = reinterpret_cast<const uint32_t*>(&lds[cur][0][0])[tid];
}

// Throughput-sized narrow trees (more climb workgroups than CUs): the bottom k + 1 levels first, one
// thread per level-k node hashing its whole subtree (width^k + ... + 1 nodes, one lane each, no LDS, no
// barriers: the fewest instructions per node), then the climb kernel on level k as its leaves, with k
// the smallest that leaves it one workgroup per CU (1M leaves, width 2: k = 2, 245 workgroups).
template <int H, int W>
__global__ __launch_bounds__(256) void merkle_subtree_kernel(const uint8_t* __restrict__ leaves, uint64_t n, int w,
                                                             uint8_t* __restrict__ tree, const TreeLevels t, int k) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t width = W ? W : static_cast<uint64_t>(w);
    if (blockIdx.x == 0 && threadIdx.x <= static_cast<uint32_t>(k)) {  // count records of levels 0..k
        uint32_t* e = reinterpret_cast<uint32_t*>(tree + 32ull * t.pos[threadIdx.x]);
        e[0] = bswap32(static_cast<uint32_t>(t.cnt[threadIdx.x]));
#pragma unroll
        for (int q = 1; q < 8; ++q) e[q] = 0;
    }
    if (i >= t.cnt[k]) return;
    uint64_t span = 1;  // level-l nodes under one level-k node
    for (int l = 0; l < k; ++l) span *= width;
    for (int l = 0; l <= k; ++l) {
        const uint8_t* in = l == 0 ? leaves : tree + 32ull * (t.pos[l - 1] + 1);
        const uint64_t nin = l == 0 ? n : t.cnt[l - 1];
        const uint64_t lo = i * span, hi = (i + 1) * span < t.cnt[l] ? (i + 1) * span : t.cnt[l];
        for (uint64_t j = lo; j < hi; ++j) {  // (this thread's own stores of level l - 1 precede these reads)
            const uint64_t first = j * width;
            const uint32_t c = static_cast<uint32_t>(nin - first < width ? nin - first : width);
            uint32_t d[8];
            hash_nodes<H>(in + 32ull * first, c, d);
            store_digest(H, tree + 32ull * (t.pos[l] + 1 + j), d);
        }
        span /= width;
    }
}

static constexpr uint64_t kClimbMaxWgs = 4096;  // level-1 workgroups up to which the four-wave path runs
static constexpr int kClimbMaxWidth = 4;  // widths the four-wave path takes at latency sizes (wider: the one-wave one)

// returns 1 when it does not apply (too many counters or workgroups, no counter slot)
static int launch_merkle_climb(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                               uint8_t* d_root, const TreeLevels& t0, hipStream_t st, bool sm3x = false) {
    ClimbTree f{};
    f.B = 1;
    f.kin = 0;
    while (f.B * width <= 256) {
        f.B *= width;
        ++f.kin;
    }
    // more workgroups than CUs: the subtree kernel first for levels 0..k (width^k <= 64 level-0 nodes per
    // thread), so that the climb kernel starts with one workgroup per CU
    const uint64_t cus = static_cast<uint64_t>(cu_count());
    // A/B hooks (read once): BCOSGPU_MERKLE_NOSUB=1 never runs the subtree kernel first (the climb kernel
    // takes the leaves itself, two workgroups on some CUs); BCOSGPU_MERKLE_LATSCHED=1 keeps the latency
    // schedule (25-lane groups from eight nodes down) even with more workgroups than CUs
    static const bool nosub_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_NOSUB");
        return e && e[0] == '1';
    }();
    static const bool latsched_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_LATSCHED");
        return e && e[0] == '1';
    }();
    int k = -1;
    if (!nosub_env && (t0.cnt[0] + f.B - 1) / f.B > cus) {
        uint64_t span = 1;
        for (int q = 0; q + 2 < t0.nlev && span <= 64; ++q, span *= width)
            if ((t0.cnt[q + 1] + f.B - 1) / f.B <= cus) {
                k = q;
                break;
            }
    }
    TreeLevels t = t0;  // the climb kernel's levels: those above level k, whose nodes are its leaves
    if (k >= 0) {
        t.nlev = t0.nlev - (k + 1);
        for (int l = 0; l < t.nlev; ++l) {
            t.pos[l] = t0.pos[l + k + 1];
            t.cnt[l] = t0.cnt[l + k + 1];
        }
    }
    f.t = t;
    // width^(g - 1) <= 8 (SM3: 64) first-level nodes per step, and the step's width^g gathered children
    // fit one LDS half (lds[0], 256 nodes): the step's first level writes lds[1] while reading them
    f.g = 1;
    for (int q = width; q <= (hasher == KECCAK256 ? 8 : 64) && q * width <= 256; q *= width) ++f.g;
    const uint64_t wgs = (t.cnt[0] + f.B - 1) / f.B;
    if (wgs > kClimbMaxWgs) return 1;
    // one workgroup per CU: the latency schedule (25-lane groups from eight nodes down, lane pairs above,
    // one lane per node only for level 1's 256); more: every SIMD runs several waves, so each level takes
    // the fewest wave-cycles -- one lane per node (a wave pass of 64 nodes: 22k cycles) down to 64 nodes,
    // lane pairs (32 nodes: 15k) down to 4, 25-lane groups (2 nodes: 9.4k) below
    const bool latency = wgs <= static_cast<uint64_t>(cu_count()) || latsched_env;
    f.coop_max = latency ? 8u : 2u;
    f.pair_max = latency ? 128u : 32u;
    f.pair = 1;
    uint32_t off = 0;
    for (int l = 0; l < t.nlev; ++l) {
        f.ctr_off[l] = off;
        if (l > f.kin) off += static_cast<uint32_t>(t.cnt[l]);
    }
    if (off > kFusedCounters) return 1;
    uint32_t* ctr = fused_counter_slot(st);
    if (!ctr) return 1;
    if (k >= 0) {
        const dim3 gs(grid_for(t0.cnt[k], 256)), bs(256);
#define SUB(HH, WW) hipLaunchKernelGGL((merkle_subtree_kernel<HH, WW>), gs, bs, 0, st, d_leaves, n, width, d_tree, t0, k)
        if (hasher == SM3) {
            if (width == 2) SUB(SM3, 2); else if (width == 16) SUB(SM3, 16); else SUB(SM3, 0);
        } else {
            if (width == 2) SUB(KECCAK256, 2); else if (width == 16) SUB(KECCAK256, 16); else SUB(KECCAK256, 0);
        }
#undef SUB
        d_leaves = d_tree + 32ull * (t0.pos[k] + 1);
        n = t0.cnt[k];
    }
    const dim3 g(static_cast<unsigned>(wgs)), b(256);
#define CLIMB(HH, WW) hipLaunchKernelGGL((merkle_climb_kernel<HH, WW>), g, b, 0, st, d_leaves, n, width, d_tree, f, d_root, ctr)
#define CLIMBX(HH, WW) hipLaunchKernelGGL((merkle_climb_kernel<HH, WW, true>), g, b, 0, st, d_leaves, n, width, d_tree, f, d_root, ctr)
    if (hasher == SM3 && sm3x && width > 2 && latency) {
        if (width == 16) CLIMBX(SM3, 16); else CLIMBX(SM3, 0);
    } else if (hasher == SM3) {
        if (width == 2) CLIMB(SM3, 2); else if (width == 16) CLIMB(SM3, 16); else CLIMB(SM3, 0);
    } else {
        if (width == 2) CLIMB(KECCAK256, 2); else if (width == 16) CLIMB(KECCAK256, 16); else CLIMB(KECCAK256, 0);
    }
#undef CLIMB
#undef CLIMBX
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

static constexpr uint64_t kTopKernelMaxIn = 16384;  // inputs per level the single-workgroup kernel takes
static constexpr uint64_t kPairMaxNodes = 32768;    // level-1 nodes up to which Keccak levels use lane pairs

int launch_merkle_levelwise(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                            uint8_t* d_root, hipStream_t st);

int launch_merkle(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                  uint8_t* d_root, hipStream_t st) {
    if (n == 0 || width < 2 || width > 64) return BCOSGPU_E_ARG;
    // A/B switch to the one-launch-per-level path, read once per process
    static const bool levelwise = [] {
        const char* lw = getenv("BCOSGPU_MERKLE_LEVELWISE");
        return lw && atoi(lw) == 1;
    }();
    if (levelwise) return launch_merkle_levelwise(hasher, width, d_leaves, n, d_tree, d_root, st);
    if (n == 1) {  // Merkle.h:177-182
        hipLaunchKernelGGL(copy32_kernel, dim3(1), dim3(64), 0, st, d_leaves, d_tree);
        if (d_root) hipLaunchKernelGGL(copy32_kernel, dim3(1), dim3(64), 0, st, d_leaves, d_root);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
    TreeLevels t{};
    uint64_t pos = 0;
    for (uint64_t m = n; m > 1;) {
        if (t.nlev >= 64) return BCOSGPU_E_ARG;
        m = (m + width - 1) / width;
        t.pos[t.nlev] = pos;
        t.cnt[t.nlev] = m;
        pos += m + 1;
        ++t.nlev;
    }
    // latency-sized trees: one launch, one wave per workgroup (BCOSGPU_MERKLE_FUSED=0/1 forces it off/on)
    static const int fused_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_FUSED");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    // narrow Keccak trees: the four-wave one-launch kernel (BCOSGPU_MERKLE_CLIMB=0/1 forces it off/on)
    static const int climb_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_CLIMB");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    // Throughput-sized trees (more level-1 nodes than 256 per CU), where the subtree kernel runs first,
    // take it at every width up to 16 and both hashers (16M leaves, width 16: Keccak 0.62 vs 0.94 ms on
    // the two-launch path, SM3 0.56 vs 0.71, profiles/r04_merkle_paths_ab_w16.json); at latency sizes
    // only narrow Keccak trees (SM3's one-lane levels measured no faster than the two-launch path,
    // profiles/r04_merkle_paths_ab_sm3.json; width 16 has the one-wave kernel)
    const bool big = t.cnt[0] > 256ull * static_cast<uint64_t>(cu_count());
    // SM3 trees of width > 2 at latency sizes (C1: 100k leaves, width 16) on the climb kernel with expanded
    // blocks -- one launch instead of merkle_wg_kernel + merkle_top_kernel -- measured no faster (C1 SM3
    // 0.1058 vs 0.1038 ms, profiles/r06_merkle_sm3_climbx_ab.json: the critical path is 38 serial
    // compressions either way, and the second launch's gap is a few us), so it is opt-in
    // (BCOSGPU_MERKLE_SM3CLIMB=1, read once)
    static const bool sm3climb_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_SM3CLIMB");
        return e && e[0] == '1';
    }();
    const bool sm3_climb = hasher == SM3 && width > 2 && !big && sm3climb_env;
    if (fused_env != 1 &&
        (climb_env == 1 || sm3_climb ||
         (climb_env < 0 && ((width <= kClimbMaxWidth && (hasher == KECCAK256 || big)) || (width <= 16 && big))))) {
        const int rc = launch_merkle_climb(hasher, width, d_leaves, n, d_tree, d_root, t, st, sm3_climb);
        if (rc <= 0) return rc;
    }
    if (fused_env == 1 || (fused_env < 0 && hasher == KECCAK256)) {
        const int rf = launch_merkle_fused(hasher, width, d_leaves, n, d_tree, d_root, t, fused_env == 1, st);
        if (rf <= 0) return rf;
    }
    int kin = 0;
    uint32_t B = 1;
    while (B * static_cast<uint32_t>(width) <= 256u) {
        B *= width;
        ++kin;
    }
    const dim3 g1(static_cast<unsigned>((t.cnt[0] + B - 1) / B));
    // Keccak levels on lane pairs while level 1 is latency-sized: at most one pair per lane of a wave
    // per SIMD (kPairMaxNodes); beyond that one lane per node, which issues fewer instructions per node.
    // BCOSGPU_MERKLE_PAIR=0/1 forces it off/on (A/B), read once per process.
    static const int pair_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_PAIR");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    const int pair = hasher == KECCAK256 && (pair_env >= 0 ? pair_env : t.cnt[0] <= kPairMaxNodes) ? 1 : 0;
    // Keccak: enough 32-lane groups that the second level runs one cooperative pass (B / width nodes),
    // two lanes per level-1 node in pair mode
    uint32_t threads = pair ? 2u * B : B;
    if (hasher == KECCAK256 && kin >= 1 && 32u * (B / width) > threads && 32u * (B / width) <= 512u) threads = 32u * (B / width);
    const dim3 b1(threads);
    // SM3 at latency sizes (a workgroup per CU at most): the LDS levels' and the top kernel's blocks
    // expanded in parallel (sm3_level_x; its 70 KB of LDS would cost a throughput-sized level 1 occupancy).
    // BCOSGPU_MERKLE_SM3X=0/1 forces it off/on (A/B), read once per process.
    static const int sm3x_env = [] {
        const char* e = getenv("BCOSGPU_MERKLE_SM3X");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    const bool sm3x = hasher == SM3 && (sm3x_env >= 0 ? sm3x_env == 1 : g1.x <= static_cast<unsigned>(cu_count()));
    const bool sm3x_top = hasher == SM3 && sm3x_env != 0;
#define WG(HH, WW, XX) hipLaunchKernelGGL((merkle_wg_kernel<HH, WW, XX>), g1, b1, 0, st, d_leaves, n, width, kin, static_cast<int>(B), d_tree, t, d_root, pair)
    if (hasher == SM3) {
        if (sm3x) {
            if (width == 2) WG(SM3, 2, true); else if (width == 16) WG(SM3, 16, true); else WG(SM3, 0, true);
        } else {
            if (width == 2) WG(SM3, 2, false); else if (width == 16) WG(SM3, 16, false); else WG(SM3, 0, false);
        }
    } else {
        if (width == 2) WG(KECCAK256, 2, false); else if (width == 16) WG(KECCAK256, 16, false); else WG(KECCAK256, 0, false);
    }
#undef WG
    int l = kin + 1;  // next level (0-based) to compute
    while (l < t.nlev && t.cnt[l - 1] > kTopKernelMaxIn) {  // wide middle levels: one launch each
        launch_level(hasher, width, d_tree + 32ull * (t.pos[l - 1] + 1), t.cnt[l - 1], d_tree + 32ull * (t.pos[l] + 1),
                     t.cnt[l], st);
        ++l;
    }
    if (l < t.nlev) {
#define TOP(HH, WW, XX) hipLaunchKernelGGL((merkle_top_kernel<HH, WW, XX>), dim3(1), dim3(1024), 0, st, width, l, d_tree, t, d_root, pair)
        if (hasher == SM3) {
            if (sm3x_top) {
                if (width == 2) TOP(SM3, 2, true); else if (width == 16) TOP(SM3, 16, true); else TOP(SM3, 0, true);
            } else {
                if (width == 2) TOP(SM3, 2, false); else if (width == 16) TOP(SM3, 16, false); else TOP(SM3, 0, false);
            }
        } else {
            if (width == 2) TOP(KECCAK256, 2, false); else if (width == 16) TOP(KECCAK256, 16, false); else TOP(KECCAK256, 0, false);
        }
#undef TOP
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_merkle_levelwise(int hasher, int width, const uint8_t* d_leaves, uint64_t n, uint8_t* d_tree,
                            uint8_t* d_root, hipStream_t st) {
    if (n == 0 || width < 2 || width > 64) return BCOSGPU_E_ARG;
    if (n == 1) {
        hipLaunchKernelGGL(copy32_kernel, dim3(1), dim3(64), 0, st, d_leaves, d_tree);
        if (d_root) hipLaunchKernelGGL(copy32_kernel, dim3(1), dim3(64), 0, st, d_leaves, d_root);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
    LevelTable t{};
    uint64_t pos = 0, nin = n;
    const uint8_t* in = d_leaves;
    while (nin > 1) {
        const uint64_t nout = (nin + width - 1) / width;
        if (t.nlevels >= 64) return BCOSGPU_E_ARG;
        t.pos[t.nlevels] = pos;
        t.count[t.nlevels] = static_cast<uint32_t>(nout);
        ++t.nlevels;
        uint8_t* out = d_tree + 32 * (pos + 1);
        launch_level(hasher, width, in, nin, out, nout, st);
        in = out;
        pos += nout + 1;
        nin = nout;
    }
    hipLaunchKernelGGL(merkle_counts_kernel, dim3(1), dim3(64), 0, st, d_tree, t);
    if (d_root) hipLaunchKernelGGL(copy32_kernel, dim3(1), dim3(64), 0, st, d_tree + 32 * (pos - 1), d_root);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

// `levels` Merkle levels of a shard whose first leaf index is a multiple of width^levels: the
// shard's level-`levels` nodes are exactly the reference tree's nodes over that range (Merkle.h
// groups every level from index 0).  Intermediate levels ping-pong through d_work
// (>= 32 * ceil(n / width) bytes); the last level lands in d_out.
int launch_merkle_levels(int hasher, int width, const uint8_t* d_in, uint64_t n, int levels, uint8_t* d_work,
                         uint8_t* d_out, hipStream_t st) {
    if (n == 0 || width < 2 || width > 64 || levels < 1) return BCOSGPU_E_ARG;
    const uint8_t* in = d_in;
    uint64_t nin = n;
    const uint64_t half = 32 * ((n + width - 1) / width);
    for (int l = 0; l < levels; ++l) {
        const uint64_t nout = (nin + width - 1) / width;
        uint8_t* out = (l + 1 == levels) ? d_out : d_work + ((l & 1) ? half : 0);
        launch_level(hasher, width, in, nin, out, nout, st);
        in = out;
        nin = nout;
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

// ------------------------------------------------------------------ many blocks' roots at once
// BlockImpl::calculateTransactionRoot / calculateReceiptRoot (BlockImpl.h:111-183) for a batch of
// blocks (sync catch-up, PBFT replay): every level of up to kSegBlocks independent trees is ONE
// launch, one output node per lane.  A block whose tree is already a single node passes it through
// (so all trees end on the same launch, and the last launch writes the roots in place); an empty
// block yields the zero hash (BlockImpl.h:114-119).
static constexpr int kSegBlocks = 64;
struct SegLevel {
    uint64_t in_off[kSegBlocks];       // first input node of block b, in 32-byte entries
    uint32_t n_in[kSegBlocks];         // input nodes of block b at this level (0 = empty block)
    uint32_t out_off[kSegBlocks + 1];  // prefix of output nodes per block
    uint32_t nb;
};

template <int H, int W>
__global__ __launch_bounds__(256) void merkle_seg_level_kernel(const uint8_t* __restrict__ in, int w,
                                                               uint8_t* __restrict__ out, const SegLevel t) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= t.out_off[t.nb]) return;
    int lo = 0, hi = static_cast<int>(t.nb) - 1;  // last b with out_off[b] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (t.out_off[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    const uint32_t j = i - t.out_off[lo], nin = t.n_in[lo];
    uint32_t* dst = reinterpret_cast<uint32_t*>(out + 32ull * i);
    if (nin <= 1u) {  // empty block -> zero hash; finished tree -> pass the root through
        const uint32_t* src = reinterpret_cast<const uint32_t*>(in + 32ull * t.in_off[lo]);
#pragma unroll
        for (int k = 0; k < 8; ++k) dst[k] = nin ? src[k] : 0u;
        return;
    }
    const uint32_t width = W ? W : static_cast<uint32_t>(w);
    const uint32_t first = j * width;
    const uint32_t cnt = (nin - first) < width ? (nin - first) : width;
    const uint32_t len = cnt * 32u;
    NodeReader rd(in + 32ull * (t.in_off[lo] + first), len);
    uint32_t d[8];
    if (H == KECCAK256) keccak256_msg(rd, len, d);
    else sm3_msg(rd, len, d);
    store_digest(H, out + 32ull * i, d);
}

uint64_t merkle_roots_work_bytes(uint64_t total_leaves, uint64_t nblocks, int width) {
    return 64ull * ((total_leaves + width - 1) / width + nblocks);
}

int launch_merkle_roots_batch(int hasher, int width, const uint8_t* d_leaves, const uint64_t* block_off,
                              uint64_t nblocks, uint8_t* d_work, uint8_t* d_roots, hipStream_t st) {
    if (width < 2 || width > 64) return BCOSGPU_E_ARG;
    if (nblocks == 0) return 0;
    const uint64_t total = block_off[nblocks] - block_off[0];
    const uint64_t half = 32ull * ((total + width - 1) / width + nblocks);  // ping-pong halves
    for (uint64_t c0 = 0; c0 < nblocks; c0 += kSegBlocks) {
        const uint32_t nb = static_cast<uint32_t>(nblocks - c0 < kSegBlocks ? nblocks - c0 : kSegBlocks);
        uint64_t cnt[kSegBlocks];
        int L = 1;
        for (uint32_t b = 0; b < nb; ++b) {
            cnt[b] = block_off[c0 + b + 1] - block_off[c0 + b];
            if (cnt[b] > 0xFFFFFFFFull) return BCOSGPU_E_ARG;
            int l = 0;
            for (uint64_t m = cnt[b]; m > 1; m = (m + width - 1) / width) ++l;
            if (l > L) L = l;
        }
        const uint8_t* in = d_leaves;
        SegLevel t{};
        t.nb = nb;
        for (uint32_t b = 0; b < nb; ++b) t.in_off[b] = block_off[c0 + b] - block_off[0];
        for (int l = 0; l < L; ++l) {
            uint32_t o = 0;
            for (uint32_t b = 0; b < nb; ++b) {
                t.n_in[b] = static_cast<uint32_t>(cnt[b]);
                t.out_off[b] = o;
                cnt[b] = cnt[b] <= 1 ? 1 : (cnt[b] + width - 1) / width;
                o += static_cast<uint32_t>(cnt[b]);
            }
            t.out_off[nb] = o;
            uint8_t* out = (l + 1 == L) ? d_roots + 32ull * c0 : d_work + ((l & 1) ? half : 0);
            dim3 g(grid_for(o, 256)), blk(256);
#define SEG(HH, WW) hipLaunchKernelGGL((merkle_seg_level_kernel<HH, WW>), g, blk, 0, st, in, width, out, t)
            if (hasher == SM3) {
                if (width == 2) SEG(SM3, 2); else if (width == 16) SEG(SM3, 16); else SEG(SM3, 0);
            } else {
                if (width == 2) SEG(KECCAK256, 2); else if (width == 16) SEG(KECCAK256, 16); else SEG(KECCAK256, 0);
            }
#undef SEG
            in = out;
            for (uint32_t b = 0; b < nb; ++b) t.in_off[b] = t.out_off[b];
        }
    }
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

// ------------------------------------------------------------------ Merkle proofs
// Merkle<H,width>::generateMerkleProof(originHashes, merkle, index, out) (Merkle.h:121-168) for a
// batch of leaf indices: one proof per lane, gathered from the leaves and the reference-layout tree.
// Proof = per level below the root: a count record (BE u32 in a 32-byte entry) and the group of
// <= width siblings that contains the node; a 1-leaf tree's proof is the single leaf.
struct ProofLevels {
    uint64_t pos[64];    // tree entry of level l's count record (level 0 = leaves: unused)
    uint64_t len[64];    // nodes at level l (level 0 = n)
    int nlev;            // levels below the root
};

__device__ __forceinline__ void copy_entry(uint8_t* dst, const uint8_t* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = s[0];
    d[1] = s[1];
}

__global__ __launch_bounds__(256) void merkle_proof_kernel(const uint8_t* __restrict__ leaves, const uint8_t* __restrict__ tree,
                                                           int width, const ProofLevels t, const uint64_t* __restrict__ index,
                                                           uint64_t m, uint64_t stride, uint8_t* __restrict__ proofs,
                                                           uint32_t* __restrict__ plen) {
    const uint64_t q = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q >= m) return;
    uint8_t* out = proofs + 32ull * stride * q;
    uint64_t idx = index[q];
    if (t.nlev == 0) {  // n == 1 (Merkle.h:137-142)
        copy_entry(out, tree);
        plen[q] = 1;
        return;
    }
    uint32_t e = 0;
    idx -= idx % width;  // indexAlign (Merkle.h:211)
    for (int l = 0; l < t.nlev; ++l) {
        const uint64_t len = t.len[l];
        const uint64_t cnt = (len - idx) < static_cast<uint64_t>(width) ? (len - idx) : static_cast<uint64_t>(width);
        uint32_t* rec = reinterpret_cast<uint32_t*>(out + 32ull * e);
        rec[0] = bswap32(static_cast<uint32_t>(cnt));
#pragma unroll
        for (int k = 1; k < 8; ++k) rec[k] = 0;
        ++e;
        const uint8_t* src = l == 0 ? leaves + 32ull * idx : tree + 32ull * (t.pos[l] + 1 + idx);
        for (uint64_t j = 0; j < cnt; ++j) copy_entry(out + 32ull * (e + j), src + 32ull * j);
        e += static_cast<uint32_t>(cnt);
        idx /= width;
        idx -= idx % width;
    }
    plen[q] = e;
}

// verifyMerkleProof(proof, hash, root) (Merkle.h:45-81), one proof per lane.  ok = 1 / 0, or 2 for an
// empty proof (the reference throws std::invalid_argument{"Empty input proof!"}).  A count record
// that runs past the proof is "false" (the reference reads out of range there).
template <int H>
__global__ __launch_bounds__(256) void merkle_verify_kernel(const uint8_t* __restrict__ proofs, uint64_t stride,
                                                            const uint32_t* __restrict__ plen,
                                                            const uint8_t* __restrict__ hashes,
                                                            const uint8_t* __restrict__ roots, int root_stride,
                                                            uint64_t m, uint8_t* __restrict__ ok) {
    const uint64_t q = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q >= m) return;
    const uint8_t* pr = proofs + 32ull * stride * q;
    const uint32_t len = plen[q] < stride ? plen[q] : static_cast<uint32_t>(stride);
    if (plen[q] == 0) {
        ok[q] = 2;
        return;
    }
    uint32_t h[8];
    const uint32_t* hs = reinterpret_cast<const uint32_t*>(hashes + 32ull * q);
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = hs[k];
    bool good = plen[q] <= stride;
    if (len > 1) {
        uint32_t it = 0;
        while (good && it < len) {
            const uint32_t cnt = bswap32(reinterpret_cast<const uint32_t*>(pr + 32ull * it)[0]);
            ++it;
            if (cnt > len - it) {
                good = false;
                break;
            }
            bool found = false;
            for (uint32_t j = 0; j < cnt; ++j) {
                const uint32_t* en = reinterpret_cast<const uint32_t*>(pr + 32ull * (it + j));
                bool eq = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) eq = eq && en[k] == h[k];
                found = found || eq;
            }
            if (!found) {
                good = false;
                break;
            }
            const uint32_t bytes = cnt * 32u;
            AlignedReader rd(pr + 32ull * it, bytes);
            uint32_t d[8];
            if (H == KECCAK256) keccak256_msg(rd, bytes, d);
            else sm3_msg(rd, bytes, d);
            uint8_t tmp[32];
            store_digest(H, tmp, d);
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = reinterpret_cast<const uint32_t*>(tmp)[k];
            it += cnt;
        }
    }
    const uint32_t* rt = reinterpret_cast<const uint32_t*>(roots + 32ull * (root_stride ? q : 0));
#pragma unroll
    for (int k = 0; k < 8; ++k) good = good && h[k] == rt[k];
    ok[q] = good ? 1 : 0;
}

uint64_t merkle_proof_stride(uint64_t n, int width) {
    if (n <= 1) return 1;
    uint64_t s = 0;
    for (uint64_t len = n; len > 1; len = (len + width - 1) / width) s += 1 + (len < static_cast<uint64_t>(width) ? len : width);
    return s;
}

int launch_merkle_proofs(int width, const uint8_t* d_leaves, uint64_t n, const uint8_t* d_tree, const uint64_t* d_index,
                         uint64_t m, uint8_t* d_proofs, uint32_t* d_len, hipStream_t st) {
    if (n == 0 || width < 2 || width > 64) return BCOSGPU_E_ARG;
    if (m == 0) return 0;
    ProofLevels t{};
    uint64_t pos = 0, len = n;
    while (len > 1) {
        if (t.nlev >= 64) return BCOSGPU_E_ARG;
        t.len[t.nlev] = len;
        const uint64_t next = (len + width - 1) / width;
        // level nlev's nodes are the children grouped at this step; their parents sit at tree entry pos
        // (count record) + 1 ..; for l >= 1 the nodes of level l live at the previous record's position
        t.pos[t.nlev] = t.nlev == 0 ? 0 : pos;
        if (t.nlev > 0) pos += len + 1;
        ++t.nlev;
        len = next;
    }
    hipLaunchKernelGGL(merkle_proof_kernel, dim3(grid_for(m, 256)), dim3(256), 0, st, d_leaves, d_tree, width, t, d_index, m,
                       merkle_proof_stride(n, width), d_proofs, d_len);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_merkle_verify(int hasher, const uint8_t* d_proofs, uint64_t stride, const uint32_t* d_len,
                         const uint8_t* d_hashes, const uint8_t* d_roots, int root_stride, uint64_t m, uint8_t* d_ok,
                         hipStream_t st) {
    if (m == 0) return 0;
    if (hasher == SM3)
        hipLaunchKernelGGL(merkle_verify_kernel<SM3>, dim3(grid_for(m, 256)), dim3(256), 0, st, d_proofs, stride, d_len,
                           d_hashes, d_roots, root_stride, m, d_ok);
    else
        hipLaunchKernelGGL(merkle_verify_kernel<KECCAK256>, dim3(grid_for(m, 256)), dim3(256), 0, st, d_proofs, stride,
                           d_len, d_hashes, d_roots, root_stride, m, d_ok);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

int launch_merkle_old(int hasher, const uint8_t* d_leaves, uint64_t n, uint8_t* d_scratch,
                      uint8_t* d_root, hipStream_t st) {
    // d_scratch: >= 32 * (ceil(n/16) + ceil(n/256) + ...) bytes; levels ping into it
    if (n == 0) {
        if (hasher == SM3) hipLaunchKernelGGL(hash_one_kernel<SM3>, dim3(1), dim3(64), 0, st, d_leaves, 0u, d_root);
        else hipLaunchKernelGGL(hash_one_kernel<KECCAK256>, dim3(1), dim3(64), 0, st, d_leaves, 0u, d_root);
        return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
    }
    const uint8_t* in = d_leaves;
    uint64_t nin = n, pos = 0;
    while (nin > 1) {
        const uint64_t nout = (nin + 15) / 16;
        uint8_t* out = d_scratch + 32 * pos;
        launch_level(hasher, 16, in, nin, out, nout, st);
        in = out;
        pos += nout;
        nin = nout;
    }
    if (hasher == SM3) hipLaunchKernelGGL(hash_one_kernel<SM3>, dim3(1), dim3(64), 0, st, in, 32u, d_root);
    else hipLaunchKernelGGL(hash_one_kernel<KECCAK256>, dim3(1), dim3(64), 0, st, in, 32u, d_root);
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}

}  // namespace bcosgpu

namespace bcosgpu {
// ------------------------------------------------------------------ the vector<bytes> tree layout
// BlockImpl::calculateTransactionRoot stores the tree in m_inner->transactionsMerkle, a
// vector<vector<char>> (BlockImpl.h:136, tars field 9), and merkleBench fills a vector<bytes>
// (merkleBench.cpp:53-56): there setNumberToHash's resizeTo(output, 4) (Merkle.h:213-217,
// concepts/bcos-concepts/Basic.h:50-61) leaves every count record a 4-byte entry, while the nodes are
// 32 bytes.  This moves the 32-byte-entry output vector into that layout, packed: entry e goes to byte
// 32 e - 28 c(e), c(e) = count records before it, and count records keep their bytes 0..3.
uint64_t merkle_levels(uint64_t n, int width) {
    uint64_t levels = 0;
    while (n > 1) {
        n = (n + width - 1) / width;
        ++levels;
    }
    return levels;
}

__global__ __launch_bounds__(256) void merkle_compact_kernel(const uint32_t* __restrict__ tree, uint64_t entries,
                                                             uint64_t n, int width, uint32_t* __restrict__ out) {
    const uint64_t e = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= entries) return;
    uint64_t pos = 0, m = n, before = 0;
    bool record = false;
    while (m > 1) {
        m = (m + width - 1) / width;
        if (e == pos) {
            record = true;
            break;
        }
        ++before;
        if (e <= pos + m) break;
        pos += m + 1;
    }
    const uint32_t* src = tree + 8 * e;
    uint32_t* dst = out + 8 * e - 7 * before;
    if (record) {
        dst[0] = src[0];
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) dst[k] = src[k];
    }
}

int launch_merkle_compact(const uint8_t* d_tree, uint64_t n, int width, uint8_t* d_out, hipStream_t st) {
    const uint64_t entries = n == 1 ? 1 : merkle_size(n, width);
    if (entries == 0) return 0;
    hipLaunchKernelGGL(merkle_compact_kernel, dim3(static_cast<unsigned>((entries + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t*>(d_tree), entries, n, width, reinterpret_cast<uint32_t*>(d_out));
    return hipGetLastError() == hipSuccess ? 0 : BCOSGPU_E_HIP;
}
}  // namespace bcosgpu
