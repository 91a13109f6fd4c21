// ecc_kernels.hip -- placeholder until the ECC kernels land (fails loudly, never silently).
#include "engine.h"
namespace bcosgpu {
int ecc_init_tables(int) { return 0; }
int launch_secp256k1_recover(const uint8_t*, const uint8_t*, uint32_t, uint64_t, uint8_t*, uint8_t*, uint8_t*, hipStream_t) { return BCOSGPU_E_ARG; }
int launch_sm2_verify(const uint8_t*, const uint8_t*, uint32_t, uint64_t, uint8_t*, uint8_t*, hipStream_t) { return BCOSGPU_E_ARG; }
int launch_secp256k1_sign(const uint8_t*, const uint8_t*, uint64_t, uint8_t*, uint8_t*, uint8_t*, hipStream_t) { return BCOSGPU_E_ARG; }
int launch_sm2_sign(const uint8_t*, const uint8_t*, uint64_t, uint8_t*, uint8_t*, hipStream_t) { return BCOSGPU_E_ARG; }
int launch_tx_verify(int, const uint8_t*, const uint64_t*, const uint8_t*, const uint64_t*, uint64_t, uint8_t*, uint8_t*, uint8_t*, hipStream_t) { return BCOSGPU_E_ARG; }
}
