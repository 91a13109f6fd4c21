// concurrent_test.cpp -- the reference's per-transaction admission call pattern against the drop-in
// SignatureCrypto classes: T threads (TxPool's submitter pool, TxPool.h:48-49) each making K single
// SignatureCrypto::recover calls (Transaction::verify, Transaction.h:68-82), every result compared
// with the oracle's.  The engine coalesces the concurrent calls into shared launches (csrc/coalesce.hip).
//
//   concurrent_test <datafile> <threads> <calls_per_thread>
// datafile (written by tests/test_concurrent.py): "BGCT", u32 suite (0 secp256k1 / 1 SM2), u32 m,
// then m x 32 hashes, m x siglen signatures (65 / 128), m expected verdicts (1 / 0), m x 64 expected
// public keys.  Prints one JSON line; exit 0 iff every call matched.
#include <bcos_gpu_crypto.hpp>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace bcos;
using namespace bcos::crypto;

int main(int argc, char** argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s datafile threads calls_per_thread\n", argv[0]);
        return 2;
    }
    if (bcosgpu_device_count() <= 0) {
        printf("no gfx950 device\n");
        return 77;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    char magic[4];
    uint32_t suite = 0, m = 0;
    if (fread(magic, 1, 4, f) != 4 || std::memcmp(magic, "BGCT", 4) != 0 || fread(&suite, 4, 1, f) != 1 ||
        fread(&m, 4, 1, f) != 1 || m == 0)
        return 2;
    const size_t siglen = suite == 0 ? 65 : 128;
    std::vector<uint8_t> hashes(32ull * m), sigs(siglen * m), ok(m), pubs(64ull * m);
    if (fread(hashes.data(), 1, hashes.size(), f) != hashes.size() || fread(sigs.data(), 1, sigs.size(), f) != sigs.size() ||
        fread(ok.data(), 1, ok.size(), f) != ok.size() || fread(pubs.data(), 1, pubs.size(), f) != pubs.size())
        return 2;
    fclose(f);
    const int threads = atoi(argv[2]);
    const int calls = atoi(argv[3]);

    bcosgpu::ref::GpuSecp256k1Crypto k1(0);
    bcosgpu::ref::GpuSM2Crypto sm2(0);
    SignatureCrypto& crypto = suite == 0 ? static_cast<SignatureCrypto&>(k1) : static_cast<SignatureCrypto&>(sm2);
    // warm the engine (tables, staging buffers) outside the timed region
    {
        HashType h;
        std::memcpy(h.data(), hashes.data(), 32);
        try {
            crypto.recover(h, bytesConstRef(sigs.data(), siglen));
        } catch (const InvalidSignature&) {
        }
    }
    std::atomic<long> mismatches{0}, valid{0}, engine_errors{0};
    std::vector<std::thread> pool;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t] {
            for (int j = 0; j < calls; ++j) {
                const size_t i = (static_cast<size_t>(j) * threads + t) % m;
                HashType h;
                std::memcpy(h.data(), hashes.data() + 32 * i, 32);
                bool got = false;
                bool same = true;
                try {
                    PublicPtr p = crypto.recover(h, bytesConstRef(sigs.data() + siglen * i, siglen));
                    got = true;
                    same = p && p->size() == 64 && std::memcmp(p->constData(), pubs.data() + 64 * i, 64) == 0;
                } catch (const InvalidSignature&) {
                    got = false;
                } catch (const SignException& e) {
                    ++engine_errors;
                    same = false;
                }
                if (got != (ok[i] != 0) || !same) ++mismatches;
                if (got) ++valid;
            }
        });
    }
    for (auto& th : pool) th.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const long total = static_cast<long>(threads) * calls;
    printf("{\"suite\": %u, \"threads\": %d, \"calls\": %ld, \"valid\": %ld, \"mismatches\": %ld, \"engine_errors\": %ld, "
           "\"seconds\": %.4f, \"calls_per_s\": %.1f}\n",
           suite, threads, total, valid.load(), mismatches.load(), engine_errors.load(), dt, total / dt);
    return mismatches.load() == 0 ? 0 : 1;
}
