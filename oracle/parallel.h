/* parallel.h -- tiny pthread parallel-for for the oracle's CPU baseline (mirrors the reference's
 * tbb::parallel_for over contiguous ranges, Merkle.h:248, TransactionSync.cpp:516).
 * TEST INFRASTRUCTURE ONLY. */
#ifndef BCOS_ORACLE_PARALLEL_H
#define BCOS_ORACLE_PARALLEL_H
#include <stddef.h>
typedef void (*oracle_range_fn)(void* ctx, size_t lo, size_t hi);
void oracle_parallel_for(size_t n, int nthreads, oracle_range_fn fn, void* ctx);
#endif
