/*
 * bcos_gpu_wedpr.h -- the wedpr-shaped single-call shims of libbcosgpu.so declared over wedpr-crypto's
 * OWN buffer types, for reference translation units that include <wedpr-crypto/WedprCrypto.h> (which
 * defines CInputBuffer { const char* data; uintptr_t len; } and COutputBuffer { char* data; uintptr_t
 * len; }).  Include it after the wedpr header; then
 *
 *     m_verifier = bcosgpu_wedpr_sm2_verify;            // SM2Crypto.h:64-65 std::function member
 *
 * compiles as written, and the shims can replace wedpr_secp256k1_recover_public_key /
 * wedpr_secp256k1_verify at their call sites (Secp256k1Crypto.cpp:51-63, :79-93).  The symbols are
 * extern "C", so these declarations and bcos_gpu.h's bcosgpu_CInputBuffer ones name the same
 * functions; the static_asserts pin the shared layout.
 */
#ifndef BCOS_GPU_WEDPR_H
#define BCOS_GPU_WEDPR_H
#define BCOSGPU_WEDPR_TYPES 1
#include <stddef.h>
#include "bcos_gpu.h"

#ifdef __cplusplus
static_assert(sizeof(CInputBuffer) == sizeof(bcosgpu_CInputBuffer), "CInputBuffer layout");
static_assert(offsetof(CInputBuffer, data) == offsetof(bcosgpu_CInputBuffer, data), "CInputBuffer::data");
static_assert(offsetof(CInputBuffer, len) == offsetof(bcosgpu_CInputBuffer, len), "CInputBuffer::len");
static_assert(sizeof(COutputBuffer) == sizeof(bcosgpu_COutputBuffer), "COutputBuffer layout");
static_assert(offsetof(COutputBuffer, len) == offsetof(bcosgpu_COutputBuffer, len), "COutputBuffer::len");
extern "C" {
#endif
/* wedpr_secp256k1_recover_public_key (Secp256k1Crypto.cpp:79-93) */
int8_t bcosgpu_wedpr_secp256k1_recover_public_key(const CInputBuffer* hash, const CInputBuffer* sig,
                                                   COutputBuffer* pub);
/* wedpr_sm2_verify / fast_sm2_verify (SM2Crypto.h:39,64-65; fast_sm2.h:35-36) */
int8_t bcosgpu_wedpr_sm2_verify(const CInputBuffer* pub, const CInputBuffer* hash, const CInputBuffer* sig);
/* wedpr_secp256k1_verify (Secp256k1Crypto.cpp:51-63) */
int8_t bcosgpu_wedpr_secp256k1_verify(const CInputBuffer* pub, const CInputBuffer* hash, const CInputBuffer* sig);
#ifdef __cplusplus
}
#endif
#endif
