// receipt_test.cpp -- BlockImpl::calculateReceiptRoot (BlockImpl.h:156-183) through the C ABI and the C++
// adapter (include/bcos_gpu.hpp calculateReceiptRoots): receipts with logs and with / without a dataHash,
// built as bcosgpu_TransactionReceiptData views over a fixture written by tests/test_receipts.py, whose
// expected preimages, hashes and roots come from the oracle's restatement of TarsHashable.h:43-75.
// argv[1] = fixture.  The packer check runs everywhere; the GPU part exits 77 without a gfx950 device.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/bcos_gpu.hpp"

using namespace bcosgpu;

namespace {
struct Reader {
    std::vector<uint8_t> d;
    size_t at = 0;
    uint32_t u32() {
        uint32_t v;
        std::memcpy(&v, d.data() + at, 4);
        at += 4;
        return v;
    }
    uint64_t u64() {
        uint64_t v;
        std::memcpy(&v, d.data() + at, 8);
        at += 8;
        return v;
    }
    std::pair<const uint8_t*, size_t> bytes() {
        const uint32_t n = u32();
        const uint8_t* p = d.data() + at;
        at += n;
        return {p, n};
    }
};
int fails = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            ++fails;                                                   \
        }                                                              \
    } while (0)
}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    Reader r;
    {
        FILE* f = std::fopen(argv[1], "rb");
        if (!f) return 2;
        std::fseek(f, 0, SEEK_END);
        r.d.resize(std::ftell(f));
        std::fseek(f, 0, SEEK_SET);
        if (std::fread(r.d.data(), 1, r.d.size(), f) != r.d.size()) return 2;
        std::fclose(f);
    }
    if (std::memcmp(r.d.data(), "RCPT", 4) != 0) return 2;
    r.at = 4;
    const uint32_t nblocks = r.u32();
    std::vector<uint64_t> block_off(nblocks + 1);
    for (auto& b : block_off) b = r.u64();
    const size_t n = block_off[nblocks];
    // the views point into the fixture bytes; topic arrays and log arrays live in these vectors
    std::vector<std::vector<bcosgpu_Bytes>> topics;
    std::vector<std::vector<bcosgpu_LogEntry>> logs(n);
    std::vector<bcosgpu_TransactionReceiptData> rec(n);
    topics.reserve(1 << 16);
    for (size_t i = 0; i < n; ++i) {
        bcosgpu_TransactionReceiptData& x = rec[i];
        std::memset(&x, 0, sizeof x);
        x.version = static_cast<int32_t>(r.u32());
        auto g = r.bytes();
        x.gas_used = reinterpret_cast<const char*>(g.first);
        x.gas_used_len = g.second;
        auto c = r.bytes();
        x.contract_address = reinterpret_cast<const char*>(c.first);
        x.contract_address_len = c.second;
        x.status = static_cast<int32_t>(r.u32());
        auto o = r.bytes();
        x.output = o.first;
        x.output_len = o.second;
        const uint32_t nl = r.u32();
        for (uint32_t l = 0; l < nl; ++l) {
            bcosgpu_LogEntry e;
            auto a = r.bytes();
            e.address = reinterpret_cast<const char*>(a.first);
            e.address_len = a.second;
            const uint32_t nt = r.u32();
            topics.emplace_back();
            for (uint32_t t = 0; t < nt; ++t) {
                auto tb = r.bytes();
                topics.back().push_back({tb.first, tb.second});
            }
            e.topics = topics.back().empty() ? nullptr : topics.back().data();
            e.ntopics = nt;
            auto db = r.bytes();
            e.data = db.first;
            e.data_len = db.second;
            logs[i].push_back(e);
        }
        x.logs = logs[i].empty() ? nullptr : logs[i].data();
        x.nlogs = nl;
        x.block_number = static_cast<int64_t>(r.u64());
        auto h = r.bytes();
        x.data_hash = h.second ? h.first : nullptr;
        x.data_hash_len = h.second;
    }
    // expected: preimages, then per hasher (Keccak256, SM3) n hashes and nblocks roots
    std::vector<std::pair<const uint8_t*, size_t>> want_pre(n);
    for (auto& p : want_pre) p = r.bytes();
    const uint8_t* want_h[2];
    const uint8_t* want_root[2];
    for (int k = 0; k < 2; ++k) {
        want_h[k] = r.d.data() + r.at;
        r.at += 32 * n;
        want_root[k] = r.d.data() + r.at;
        r.at += 32 * nblocks;
    }
    if (r.at != r.d.size()) {
        std::printf("fixture size mismatch\n");
        return 2;
    }

    // host packer (TarsHashable.h:54-73) against the restatement's preimages
    const uint64_t total = bcosgpu_receipt_preimage_size(rec.data(), n);
    std::vector<uint8_t> packed(total + 1);
    std::vector<uint64_t> off(n + 1);
    CHECK(bcosgpu_pack_receipt_preimages(rec.data(), n, packed.data(), total, off.data()) == BCOSGPU_OK);
    for (size_t i = 0; i < n; ++i) {
        CHECK(off[i + 1] - off[i] == want_pre[i].second);
        if (off[i + 1] - off[i] == want_pre[i].second && want_pre[i].second)
            CHECK(std::memcmp(packed.data() + off[i], want_pre[i].first, want_pre[i].second) == 0);
    }
    if (total) CHECK(bcosgpu_pack_receipt_preimages(rec.data(), n, packed.data(), total - 1, off.data()) == BCOSGPU_E_ARG);
    {   // a dataHash longer than the 32-byte hash: the reference's assignTo throws NoEnoughSpace
        bcosgpu_TransactionReceiptData bad = rec[0];
        static const uint8_t long_hash[33] = {0};
        bad.data_hash = long_hash;
        bad.data_hash_len = 33;
        uint64_t o2[2];
        CHECK(bcosgpu_pack_receipt_preimages(&bad, 1, packed.data(), packed.size(), o2) == BCOSGPU_E_ARG);
    }
    if (fails) return 1;
    if (bcosgpu_device_count() <= 0 || bcosgpu_init(0) != 0) {
        std::printf("packer ok; no gfx950 device: %s\n", bcosgpu_last_error());
        return 77;
    }
    std::vector<std::vector<bcosgpu_TransactionReceiptData>> blocks(nblocks);
    for (uint32_t b = 0; b < nblocks; ++b)
        blocks[b].assign(rec.begin() + block_off[b], rec.begin() + block_off[b + 1]);
    std::vector<HashType> hashes;
    const auto rk = calculateReceiptRoots<BCOSGPU_KECCAK256>(blocks, &hashes);
    const auto rs = calculateReceiptRoots<BCOSGPU_SM3>(blocks);
    for (uint32_t b = 0; b < nblocks; ++b) {
        CHECK(std::memcmp(rk[b].data(), want_root[0] + 32 * b, 32) == 0);
        CHECK(std::memcmp(rs[b].data(), want_root[1] + 32 * b, 32) == 0);
    }
    CHECK(hashes.size() == n);
    for (size_t i = 0; i < n && hashes.size() == n; ++i) CHECK(std::memcmp(hashes[i].data(), want_h[0] + 32 * i, 32) == 0);
    // one block through calculateReceiptRoot; no receipts -> the zero hash (BlockImpl.h:159-163)
    if (nblocks) CHECK(std::memcmp(calculateReceiptRoot<BCOSGPU_SM3>(blocks[0]).data(), want_root[1], 32) == 0);
    CHECK(calculateReceiptRoot<BCOSGPU_KECCAK256>({}) == HashType{});
    if (fails) return 1;
    std::printf("receipt_test: ok (%zu receipts, %u blocks)\n", n, nblocks);
    return 0;
}
