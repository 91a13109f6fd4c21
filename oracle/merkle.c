/*
 * merkle.c -- oracle restatement of the two Merkle algorithms.  TEST INFRASTRUCTURE ONLY.
 *
 * "new": bcos::crypto::merkle::Merkle<Hasher,width>::generateMerkle
 *        (bcos-crypto/bcos-crypto/merkle/Merkle.h:170-208, calculateLevelHashes :243-261,
 *         getMerkleSize :224-236, getNextLevelSize :238-241, setNumberToHash :213-217).
 * "old": bcos::protocol::calculateMerkleProofRoot
 *        (bcos-protocol/bcos-protocol/ParallelMerkleProof.cpp:32-69, MAX_CHILD_COUNT = 16 :30).
 * Pinned by the roots the reference's own Merkle.h produced (tests/golden/merkle.json).
 */
#include "oracle.h"
#include "parallel.h"
#include <stdlib.h>
#include <string.h>

size_t oracle_merkle_size(size_t n, int width)
{
    size_t nodes = 0;
    while (n > 1) { /* Merkle.h:229-233: each level adds its nodes + 1 count record */
        n = (n + (size_t)width - 1) / (size_t)width;
        nodes += n + 1;
    }
    return nodes;
}

typedef struct {
    int hasher, width;
    const uint8_t* in;
    size_t nin;
    uint8_t* out;
} level_ctx;

static void level_range(void* p, size_t lo, size_t hi)
{
    level_ctx* c = (level_ctx*)p;
    uint8_t buf[32 * 64];
    for (size_t i = lo; i < hi; ++i) { /* Merkle.h:252-258: hash <= width consecutive children */
        size_t first = i * (size_t)c->width, last = first + (size_t)c->width;
        if (last > c->nin) last = c->nin;
        memcpy(buf, c->in + 32 * first, 32 * (last - first));
        oracle_hash(c->hasher, buf, 32 * (last - first), c->out + 32 * i);
    }
}

static void set_count(uint8_t* e, uint32_t count)
{
    memset(e, 0, 32);
    e[0] = (uint8_t)(count >> 24); e[1] = (uint8_t)(count >> 16);
    e[2] = (uint8_t)(count >> 8); e[3] = (uint8_t)count;
}

int oracle_merkle(int hasher, int width, const uint8_t* leaves, size_t n, uint8_t root[32],
                  uint8_t* levels, int nthreads)
{
    if (n == 0 || width < 2 || width > 64) return -1; /* Merkle.h:172-175 throws on empty input */
    if (n == 1) {                                   /* Merkle.h:177-182: root = the single leaf */
        memcpy(root, leaves, 32);
        if (levels) memcpy(levels, leaves, 32);
        return 0;
    }
    size_t total = oracle_merkle_size(n, width);
    uint8_t* tree = levels ? levels : (uint8_t*)malloc(32 * total);
    size_t pos = 0;
    const uint8_t* in = leaves;
    size_t nin = n;
    while (nin > 1) {
        size_t nout = (nin + (size_t)width - 1) / (size_t)width;
        set_count(tree + 32 * pos, (uint32_t)nout);
        ++pos;
        level_ctx c = {hasher, width, in, nin, tree + 32 * pos};
        oracle_parallel_for(nout, nthreads, level_range, &c);
        in = tree + 32 * pos;
        pos += nout;
        nin = nout;
    }
    memcpy(root, tree + 32 * (total - 1), 32); /* root = last element (merkleBench.cpp:58) */
    if (!levels) free(tree);
    return 0;
}

void oracle_merkle_old(int hasher, const uint8_t* leaves, size_t n, uint8_t root[32])
{
    if (n == 0) { /* ParallelMerkleProof.cpp:35-38: empty -> H("") */
        oracle_hash(hasher, (const uint8_t*)"", 0, root);
        return;
    }
    uint8_t* cur = (uint8_t*)malloc(32 * n);
    memcpy(cur, leaves, 32 * n);
    size_t nin = n;
    while (nin > 1) { /* :44-66: same width-16 grouping as "new" */
        size_t nout = (nin + 15) / 16;
        uint8_t* nxt = (uint8_t*)malloc(32 * nout);
        level_ctx c = {hasher, 16, cur, nin, nxt};
        level_range(&c, 0, nout);
        free(cur);
        cur = nxt;
        nin = nout;
    }
    oracle_hash(hasher, cur, 32, root); /* :68 extra final hash of the top node */
    free(cur);
}
