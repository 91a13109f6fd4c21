// callbench.cpp -- single-call throughput of the engine's coalesced entry points (bench.py leg
// single_call_<T>t): T host threads, each making K calls of bcosgpu_secp256k1_recover / bcosgpu_sm2_verify
// (one signature per call, the reference's per-tx SignatureCrypto::recover pattern), every result checked
// against the expected verdict and key.
//
//   callbench <datafile> <threads> <calls_per_thread> [device]
// datafile: "BGCT", u32 suite, u32 m, m x 32 hashes, m x siglen signatures (65 / 128), m verdicts,
// m x 64 keys (the format of tests/cpp/concurrent_test.cpp).  One JSON line on stdout.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <sched.h>
#include <sys/resource.h>

#include "../../include/bcos_gpu.h"

static double cpu_seconds(const rusage& r) {
    return r.ru_utime.tv_sec + r.ru_stime.tv_sec + 1e-6 * (r.ru_utime.tv_usec + r.ru_stime.tv_usec);
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s datafile threads calls_per_thread [device]\n", argv[0]);
        return 2;
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
    const int threads = atoi(argv[2]), calls = atoi(argv[3]);
    const int dev = argc > 4 ? atoi(argv[4]) : 0;
    auto one = [&](size_t i, uint8_t* pub) {
        if (suite == 0) return bcosgpu_secp256k1_recover(dev, hashes.data() + 32 * i, sigs.data() + 65 * i, 65, pub);
        return bcosgpu_sm2_verify(dev, sigs.data() + 128 * i + 64, hashes.data() + 32 * i, sigs.data() + 128 * i);
    };
    uint8_t warm[64];
    if (one(0, warm) < 0) {
        printf("{\"error\": \"%s\"}\n", bcosgpu_last_error());
        return 1;
    }
    uint64_t st[10];
    bcosgpu_coalesce_stats(dev, st, 1);  // zero the coalescer's counters: the timed calls only
    std::atomic<long> mismatches{0}, errors{0};
    std::vector<std::vector<float>> lat(threads), when(threads);  // latency, start (us since t0)
    std::vector<std::thread> pool;
    rusage ru0{}, ru1{};
    getrusage(RUSAGE_SELF, &ru0);
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t] {
            lat[t].reserve(calls);
            when[t].reserve(calls);
            uint8_t pub[64];
            for (int j = 0; j < calls; ++j) {
                const size_t i = (static_cast<size_t>(j) * threads + t) % m;
                const auto a = std::chrono::steady_clock::now();
                when[t].push_back(std::chrono::duration<float, std::micro>(a - t0).count());
                const int rc = one(i, pub);
                lat[t].push_back(std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - a).count());
                if (rc < 0) ++errors;
                else if ((rc == 1) != (ok[i] != 0) || (suite == 0 && rc == 1 && std::memcmp(pub, pubs.data() + 64 * i, 64)))
                    ++mismatches;
            }
        });
    }
    for (auto& th : pool) th.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    getrusage(RUSAGE_SELF, &ru1);
    // the host side: CPUs this process may run on, CPU time it used over the timed calls (user + sys, all
    // threads) as busy cores, and the preemptions (involuntary context switches) per call
    cpu_set_t cs;
    CPU_ZERO(&cs);
    const int cpus = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? CPU_COUNT(&cs) : -1;
    const double busy = (cpu_seconds(ru1) - cpu_seconds(ru0)) / dt;
    const double nivcsw = double(ru1.ru_nivcsw - ru0.ru_nivcsw), nvcsw = double(ru1.ru_nvcsw - ru0.ru_nvcsw);
    std::vector<float> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    const long total = static_cast<long>(threads) * calls;
    // the tail: calls slower than 4 x p50, by the tenth of the timed run they started in
    const float slow = 4.0f * all[all.size() / 2];
    long by_tenth[10] = {0};
    for (int t = 0; t < threads; ++t)
        for (size_t j = 0; j < lat[t].size(); ++j)
            if (lat[t][j] > slow) ++by_tenth[std::min(9, static_cast<int>(when[t][j] / (dt * 1e5)))];
    char tail[256];
    snprintf(tail, sizeof tail, "{\"p90\": %.1f, \"p95\": %.1f, \"p999\": %.1f, \"slow_us\": %.1f, \"slow_by_tenth\": [%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld,%ld]}",
             all[all.size() * 90 / 100], all[all.size() * 95 / 100], all[all.size() * 999 / 1000], slow, by_tenth[0],
             by_tenth[1], by_tenth[2], by_tenth[3], by_tenth[4], by_tenth[5], by_tenth[6], by_tenth[7], by_tenth[8],
             by_tenth[9]);
    bcosgpu_coalesce_stats(dev, st, 0);
    // per call: mutex wait, queue wait; per batch: leader's host work, GPU round trip, scatter; per wake-up:
    // scheduler latency (notify -> running); busy = fraction of the wall time some batch was in flight
    const double b = st[0] ? double(st[0]) : 1.0, c = st[1] ? double(st[1]) : 1.0, w = st[8] ? double(st[8]) : 1.0;
    printf("{\"suite\": %u, \"threads\": %d, \"calls\": %ld, \"seconds\": %.4f, \"calls_per_s\": %.1f, "
           "\"latency_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, \"mismatches\": %ld, \"engine_errors\": %ld, "
           "\"coalescer\": {\"batches\": %llu, \"calls_per_batch\": %.2f, \"lock_us_per_call\": %.2f, "
           "\"queue_us_per_call\": %.2f, \"lead_us_per_batch\": %.2f, \"gpu_us_per_batch\": %.2f, "
           "\"scatter_us_per_batch\": %.2f, \"wake_us\": %.2f, \"wakes_per_call\": %.2f, \"batches_in_flight\": %.3f}, "
           "\"host\": {\"cpus_allowed\": %d, \"cores_busy\": %.2f, \"cpu_us_per_call\": %.2f, "
           "\"preemptions_per_call\": %.3f, \"voluntary_switches_per_call\": %.3f}, \"tail\": %s}\n",
           suite, threads, total, dt, total / dt, all[all.size() / 2], all[all.size() * 99 / 100], all.back(),
           mismatches.load(), errors.load(), (unsigned long long)st[0], st[1] / b, st[9] / c / 1e3, st[3] / c / 1e3,
           st[4] / b / 1e3, st[5] / b / 1e3, st[6] / b / 1e3, st[7] / w / 1e3, st[8] / c, st[5] / 1e9 / dt,
           cpus, busy, busy * dt / total * 1e6, nivcsw / total, nvcsw / total, tail);
    return mismatches.load() || errors.load() ? 1 : 0;
}
