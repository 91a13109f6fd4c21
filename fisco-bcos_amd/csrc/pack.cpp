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

// ---- receipts: impl_calculate<Hasher>(bcostars::TransactionReceipt), TarsHashable.h:43-75.  A receipt
// with a dataHash is not hashed (:47-51), so its preimage is empty here.
size_t receipt_len(const bcosgpu_TransactionReceiptData& r) {
    if (r.data_hash_len) return 0;
    size_t s = 4 + r.gas_used_len + r.contract_address_len + 4 + r.output_len + 8;
    for (size_t l = 0; l < r.nlogs; ++l) {
        const bcosgpu_LogEntry& e = r.logs[l];
        s += e.address_len + e.data_len;
        for (size_t t = 0; t < e.ntopics; ++t) s += e.topics[t].len;
    }
    return s;
}

bool valid(const bcosgpu_TransactionReceiptData& r) {
    if (r.data_hash_len) return r.data_hash && r.data_hash_len <= 32;
    if ((!r.gas_used && r.gas_used_len) || (!r.contract_address && r.contract_address_len) ||
        (!r.output && r.output_len) || (!r.logs && r.nlogs))
        return false;
    for (size_t l = 0; l < r.nlogs; ++l) {
        const bcosgpu_LogEntry& e = r.logs[l];
        if ((!e.address && e.address_len) || (!e.data && e.data_len) || (!e.topics && e.ntopics)) return false;
        for (size_t t = 0; t < e.ntopics; ++t)
            if (!e.topics[t].data && e.topics[t].len) return false;
    }
    return true;
}

void be(uint8_t* o, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; ++i) o[i] = uint8_t(v >> (8 * (bytes - 1 - i)));
}

// be32(version) || gasUsed || contractAddress || be32(status) || output ||
// for each log (address || topic_0 .. topic_k || data) || be64(blockNumber)      (TarsHashable.h:54-73)
void pack_receipt(const bcosgpu_TransactionReceiptData& r, uint8_t* o) {
    if (r.data_hash_len) return;
    uint8_t w[8];
    be(w, static_cast<uint32_t>(r.version), 4);
    o = put(o, w, 4);
    o = put(o, r.gas_used, r.gas_used_len);
    o = put(o, r.contract_address, r.contract_address_len);
    be(w, static_cast<uint32_t>(r.status), 4);
    o = put(o, w, 4);
    o = put(o, r.output, r.output_len);
    for (size_t l = 0; l < r.nlogs; ++l) {
        const bcosgpu_LogEntry& e = r.logs[l];
        o = put(o, e.address, e.address_len);
        for (size_t t = 0; t < e.ntopics; ++t) o = put(o, e.topics[t].data, e.topics[t].len);
        o = put(o, e.data, e.data_len);
    }
    be(w, static_cast<uint64_t>(r.block_number), 8);
    put(o, w, 8);
}

// items [0, n) packed by `pack(i, out + offsets[i])` on a pool of std::threads over contiguous ranges
template <class F>
void pack_parallel(size_t n, F&& pack) {
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(hw, std::max<size_t>(1, n / 4096));  // threads only for large batches
    if (nt == 1) {
        for (size_t i = 0; i < n; ++i) pack(i);
        return;
    }
    std::vector<std::thread> pool;
    const size_t per = (n + nt - 1) / nt;
    for (size_t k = 0; k < nt; ++k) {
        const size_t lo = std::min(n, k * per), hi = std::min(n, (k + 1) * per);
        if (lo < hi)
            pool.emplace_back([&pack, lo, hi] {
                for (size_t i = lo; i < hi; ++i) pack(i);
            });
    }
    for (auto& th : pool) th.join();
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
    pack_parallel(n, [&](size_t i) { pack_one(txs[i], out + offsets[i]); });
    return BCOSGPU_OK;
}

uint64_t bcosgpu_receipt_preimage_size(const bcosgpu_TransactionReceiptData* receipts, size_t n) {
    if (!receipts) return 0;
    uint64_t s = 0;
    for (size_t i = 0; i < n; ++i) s += receipt_len(receipts[i]);
    return s;
}

int bcosgpu_pack_receipt_preimages(const bcosgpu_TransactionReceiptData* receipts, size_t n, uint8_t* out,
                                   uint64_t cap, uint64_t* offsets) {
    if (n == 0) {
        if (offsets) offsets[0] = 0;
        return BCOSGPU_OK;
    }
    if (!receipts || !offsets) return BCOSGPU_E_ARG;
    offsets[0] = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!valid(receipts[i])) return BCOSGPU_E_ARG;
        offsets[i + 1] = offsets[i] + receipt_len(receipts[i]);
    }
    if (offsets[n] > cap || (offsets[n] && !out)) return BCOSGPU_E_ARG;
    pack_parallel(n, [&](size_t i) { pack_receipt(receipts[i], out + offsets[i]); });
    return BCOSGPU_OK;
}

void bcosgpu_apply_receipt_data_hashes(const bcosgpu_TransactionReceiptData* receipts, size_t n, uint8_t* hashes32) {
    if (!receipts || !hashes32) return;
    for (size_t i = 0; i < n; ++i) {
        const bcosgpu_TransactionReceiptData& r = receipts[i];
        if (!r.data_hash_len || r.data_hash_len > 32 || !r.data_hash) continue;
        std::memset(hashes32 + 32 * i, 0, 32);
        std::memcpy(hashes32 + 32 * i, r.data_hash, r.data_hash_len);
    }
}

}  // extern "C"
