// multi_test.cpp -- the device-set C ABI (include/bcos_gpu.h "device sets") from C++, as a FISCO node
// process would call it: one process, a device list, a whole block verified and its tx root computed.
//
//   multi_test <datafile> <device list, e.g. 0,0>
// datafile (tests/test_multi.py): "BGMT", u32 suite, u32 n, u32 width, u64 pre_bytes, pre, (n+1) u64
// pre_off, u64 sig_bytes, sig, (n+1) u64 sig_off, then the oracle's n x 32 tx hashes, n x 20 senders,
// n statuses and the 32-byte width-`width` root over the tx hashes.  Checks, against those:
//   bcosgpu_block_verify_multi (verdicts + root), bcosgpu_tx_verify_batch_multi,
//   bcosgpu_merkle_root_multi over the oracle's hashes, bcosgpu_secp256k1_recover_batch_multi /
//   bcosgpu_sm2_verify_batch_multi (ok = status == 0).  Prints "multi_test: ok"; exit 1 on a mismatch,
//   77 without a GPU.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bcos_gpu.h"

template <class T>
static bool rd(FILE* f, std::vector<T>& v, size_t n) {
    v.resize(n);
    return fread(v.data(), sizeof(T), n, f) == n;
}

static int fail(const char* what) {
    printf("multi_test: FAIL %s (%s)\n", what, bcosgpu_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s datafile devices\n", argv[0]);
        return 2;
    }
    if (bcosgpu_device_count() <= 0) {
        printf("multi_test: no GPU\n");
        return 77;
    }
    std::vector<int> devs;
    for (const char* p = argv[2]; *p;) {
        devs.push_back(atoi(p));
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    char magic[4];
    uint32_t hdr[3];
    uint64_t pb = 0, sb = 0;
    std::vector<uint8_t> pre, sig, th, snd, st, root;
    std::vector<uint64_t> po, so;
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "BGMT", 4) != 0 || fread(hdr, 4, 3, f) != 3) return 2;
    const uint32_t suite = hdr[0], n = hdr[1], width = hdr[2];
    if (fread(&pb, 8, 1, f) != 1 || !rd(f, pre, pb) || !rd(f, po, n + 1) || fread(&sb, 8, 1, f) != 1 || !rd(f, sig, sb) ||
        !rd(f, so, n + 1) || !rd(f, th, 32ull * n) || !rd(f, snd, 20ull * n) || !rd(f, st, n) || !rd(f, root, 32))
        return 2;
    fclose(f);
    const int nd = static_cast<int>(devs.size());
    if (bcosgpu_init_devices(devs.data(), nd) != 0) return fail("init_devices");

    std::vector<uint8_t> gh(32ull * n), gs(20ull * n), gst(n), groot(32);
    if (bcosgpu_block_verify_multi(devs.data(), nd, suite, pre.data(), po.data(), sig.data(), so.data(), n, width,
                                   gh.data(), gs.data(), gst.data(), groot.data()) != 0)
        return fail("block_verify_multi");
    if (gh != th) return fail("block_verify_multi tx hashes");
    if (gs != snd) return fail("block_verify_multi senders");
    if (gst != st) return fail("block_verify_multi statuses");
    if (groot != root) return fail("block_verify_multi root");

    std::fill(gst.begin(), gst.end(), 0xee);
    if (bcosgpu_tx_verify_batch_multi(devs.data(), nd, suite, pre.data(), po.data(), sig.data(), so.data(), n, gh.data(),
                                      gs.data(), gst.data()) != 0 || gst != st || gh != th)
        return fail("tx_verify_batch_multi");

    std::fill(groot.begin(), groot.end(), 0);
    if (bcosgpu_merkle_root_multi(devs.data(), nd, suite == 0 ? BCOSGPU_KECCAK256 : BCOSGPU_SM3, width, th.data(), n,
                                  groot.data()) != 0 || groot != root)
        return fail("merkle_root_multi");

    // the signature batches: rebuild (hash, sig) rows from the tx batch (fixed-length signatures only)
    const size_t sl = suite == 0 ? 65 : 128;
    std::vector<uint8_t> sigs(sl * n), ok(n, 0xee);
    bool fixed = true;
    for (uint32_t i = 0; i < n; ++i) {
        if (so[i + 1] - so[i] != sl) {
            fixed = false;
            break;
        }
        memcpy(sigs.data() + sl * i, sig.data() + so[i], sl);
    }
    if (fixed) {
        const int rc = suite == 0 ? bcosgpu_secp256k1_recover_batch_multi(devs.data(), nd, th.data(), sigs.data(), n,
                                                                            nullptr, nullptr, ok.data())
                                  : bcosgpu_sm2_verify_batch_multi(devs.data(), nd, th.data(), sigs.data(), n, nullptr,
                                                                   ok.data());
        if (rc != 0) return fail("signature batch multi");
        for (uint32_t i = 0; i < n; ++i)
            if ((ok[i] != 0) != (st[i] == 0)) return fail("signature batch multi verdicts");
    }
    printf("multi_test: ok (n = %u, %d shards)\n", n, nd);
    return 0;
}
