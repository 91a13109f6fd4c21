// tars_host.cpp -- host build of the Tars transaction decoder (csrc/tars_decode.h, the exact code the
// decode kernel runs), for the CPU test suite: tests/test_tars.py fuzzes it against oracle/tars.py.
// Test tool only; nothing in the product path loads it.
#include "../csrc/tars_decode.h"

using namespace bcosgpu::tars;

// per tx i: ok[i]; spans[i * 2 F_N + 2 k] / [.. + 1] = offset / length of field k (F_CHAIN .. F_HASH);
// ints[2 i] = version, ints[2 i + 1] = blockLimit
extern "C" int tars_host_decode(const uint8_t* enc, const uint64_t* off, uint64_t n, uint64_t* spans, int64_t* ints,
                                uint8_t* ok) {
    for (uint64_t i = 0; i < n; ++i) {
        TxFields f;
        ok[i] = decode_tx(enc, off[i], off[i + 1], f) ? 1 : 0;
        for (int k = 0; k < F_N; ++k) {
            spans[i * 2 * F_N + 2 * k] = f.off[k];
            spans[i * 2 * F_N + 2 * k + 1] = f.len[k];
        }
        ints[2 * i] = f.version;
        ints[2 * i + 1] = f.block_limit;
    }
    return F_N;
}
