// pack.cpp -- host-side zero-copy packer of tx-hash preimages into the SoA layout the kernels read
// (SURVEY.md §8(f)3).  Field order and encodings restate impl_calculate<Hasher>(bcostars::Transaction)
// (bcos-tars-protocol/bcos-tars-protocol/impl/TarsHashable.h:16-41): be32(version) || chainID ||
// groupID || be64(blockLimit) || nonce || to || input || abi.  Large batches are packed by a pool of
// std::threads over contiguous ranges (each range's output offset is known from a prefix sum), into
// caller memory (e.g. pinned host or HIP-registered buffers handed to bcosgpu_tx_verify_batch_dev's copy).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>
#include "../../include/bcos_gpu.h"

namespace {

size_t preimage_len(const bcosgpu_TransactionData& t) {
    return 4 + t.chain_id_len + t.group_id_len + 8 + t.nonce_len + t.to_len + t.input_len + t.abi_len;
}

uint8_t* put(uint8_t* o, const void* p, size_t n) {
    if (n) std::memcpy(o, p, n);
    return o + n;
}

void pack_one(const bcosgpu_TransactionData& t, uint8_t* o) {
    const uint32_t v = static_cast<uint32_t>(t.version);
    const uint8_t ver[4] = {uint8_t(v >> 24), uint8_t(v >> 16), uint8_t(v >> 8), uint8_t(v)};
    const uint64_t b = static_cast<uint64_t>(t.block_limit);
    uint8_t bl[8];
    for (int i = 0; i < 8; ++i) bl[i] = uint8_t(b >> (56 - 8 * i));
    o = put(o, ver, 4);
    o = put(o, t.chain_id, t.chain_id_len);
    o = put(o, t.group_id, t.group_id_len);
    o = put(o, bl, 8);
    o = put(o, t.nonce, t.nonce_len);
    o = put(o, t.to, t.to_len);
    o = put(o, t.input, t.input_len);
    put(o, t.abi, t.abi_len);
}

bool valid(const bcosgpu_TransactionData& t) {
    return (t.chain_id || !t.chain_id_len) && (t.group_id || !t.group_id_len) && (t.nonce || !t.nonce_len) &&
           (t.to || !t.to_len) && (t.input || !t.input_len) && (t.abi || !t.abi_len);
}

}  // namespace

extern "C" {

uint64_t bcosgpu_tx_preimage_size(const bcosgpu_TransactionData* txs, size_t n) {
    if (!txs) return 0;
    uint64_t s = 0;
    for (size_t i = 0; i < n; ++i) s += preimage_len(txs[i]);
    return s;
}

int bcosgpu_pack_tx_preimages(const bcosgpu_TransactionData* txs, size_t n, uint8_t* out, uint64_t cap,
                              uint64_t* offsets) {
    if (n == 0) {
        if (offsets) offsets[0] = 0;
        return BCOSGPU_OK;
    }
    if (!txs || !offsets) return BCOSGPU_E_ARG;
    offsets[0] = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!valid(txs[i])) return BCOSGPU_E_ARG;
        offsets[i + 1] = offsets[i] + preimage_len(txs[i]);
    }
    if (offsets[n] > cap || (offsets[n] && !out)) return BCOSGPU_E_ARG;
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(hw, std::max<size_t>(1, n / 4096));  // threads only for large batches
    auto work = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) pack_one(txs[i], out + offsets[i]);
    };
    if (nt == 1) {
        work(0, n);
        return BCOSGPU_OK;
    }
    std::vector<std::thread> pool;
    const size_t per = (n + nt - 1) / nt;
    for (size_t k = 0; k < nt; ++k) {
        const size_t lo = std::min(n, k * per), hi = std::min(n, (k + 1) * per);
        if (lo < hi) pool.emplace_back(work, lo, hi);
    }
    for (auto& th : pool) th.join();
    return BCOSGPU_OK;
}

}  // extern "C"
