// sigcrypto_test.cpp -- the drop-in SignatureCrypto subclasses of include/bcos_gpu_crypto.hpp, used
// through the reference's polymorphic interface (SignatureCrypto&), written like
// bcos-crypto/test/unittests/SignatureTest.cpp.  Compiled against tests/cpp/mirror/ (the interface
// shapes); exit 0 = pass, 77 = compiled and linked but no gfx950 device here.
#include <bcos_gpu_crypto.hpp>

#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

using namespace bcos;
using namespace bcos::crypto;

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);        \
            ++fails;                                                  \
        }                                                             \
    } while (0)

static bytes unhex(const char* h) {
    bytes b(strlen(h) / 2);
    for (size_t i = 0; i < b.size(); ++i) sscanf(h + 2 * i, "%2hhx", &b[i]);
    return b;
}
static HashType hash_of(const char* hex) {
    HashType h;
    bytes b = unhex(hex);
    std::memcpy(h.data(), b.data(), 32);
    return h;
}
template <class F>
static bool throws_invalid(F&& f) {
    try {
        f();
    } catch (const InvalidSignature&) {
        return true;
    }
    return false;
}
// an engine error must surface as SignException, never as InvalidSignature
template <class F>
static bool throws_sign_exception(F&& f) {
    try {
        f();
    } catch (const InvalidSignature&) {
        return false;
    } catch (const SignException&) {
        return true;
    }
    return false;
}

// Hash::hash over the engine's Keccak256 (the Hash::Ptr that recoverAddress takes)
struct GpuKeccak : Hash {
    HashType hash(bytesConstRef d) override {
        HashType h;
        uint64_t off[2] = {0, d.size()};
        static const uint8_t zero = 0;
        if (bcosgpu_keccak256_batch(d.size() ? d.data() : &zero, off, 1, h.data()) != 0) throw SignException();
        return h;
    }
};

// exposes SM2Crypto::m_verifier (SM2Crypto.h:64-65)
struct SM2Probe : bcosgpu::ref::GpuSM2Crypto {
    using bcosgpu::ref::GpuSM2Crypto::GpuSM2Crypto;
    int8_t callVerifier(const bytes& pub, const HashType& h, const bytes& sig) const {
        CInputBuffer p{(const char*)pub.data(), pub.size()}, hh{(const char*)h.data(), 32},
            s{(const char*)sig.data(), 64};
        return m_verifier(&p, &hh, &s);
    }
};

int main() {
    if (bcosgpu_device_count() <= 0) {
        printf("no gfx950 device\n");
        return 77;
    }
    bcosgpu::ref::GpuSecp256k1Crypto secp;
    bcosgpu::ref::GpuSM2Crypto sm2;
    SignatureCrypto& k1 = secp;
    SignatureCrypto& s2 = sm2;

    // ecrecover vector (EVMPrecompiledTest.cpp:58-72): recid 0, address ceaccac6...
    const char* H = "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e";
    bytes sig = unhex(H);
    bytes s = unhex("789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02");
    sig.insert(sig.end(), s.begin(), s.end());
    sig.push_back(0);
    HashType mh = hash_of(H);
    PublicPtr pub = k1.recover(mh, bytesConstRef(sig));
    CHECK(pub && pub->size() == 64);
    uint8_t d[32];
    uint64_t off[2] = {0, 64};
    CHECK(bcosgpu_keccak256_batch((const uint8_t*)pub->constData(), off, 1, d) == 0);
    static const uint8_t want[20] = {0xce, 0xac, 0xca, 0xc6, 0x40, 0xad, 0xf5, 0x5b, 0x20, 0x28,
                                     0x46, 0x9b, 0xd3, 0x6b, 0xa5, 0x01, 0xf2, 0x8b, 0x69, 0x9d};
    CHECK(std::memcmp(d + 12, want, 20) == 0);
    CHECK(k1.verify(pub, mh, bytesConstRef(sig)));  // known-key verify (Secp256k1Crypto.cpp:51-63)
    // the bytes overload: the reference calls the free secp256k1Verify (Secp256k1Crypto.cpp:126-131),
    // which the mirror makes throw -- so this passes only through the adapter's own override
    CHECK(k1.verify(std::make_shared<const bytes>(pub->data()), mh, bytesConstRef(sig)));
    CHECK(!k1.verify(std::make_shared<const bytes>(pub->data()), hash_of(
        "48bed44d1bcd124a28c27f343a817e5f5243190d3c52bf347daf876de1dbbf77"), bytesConstRef(sig)));
    // recoverAddress (Secp256k1Crypto.cpp:95-124): meant as hash || v || r || s, v = 27 / 28 -- but the
    // reference copies only sizeof(bytesConstRef) = 16 bytes into zeroed fields (:104), so v reads 0 and
    // even a valid ecrecover input gives {false, {}}; the adapter keeps that behaviour
    auto keccak = std::make_shared<GpuKeccak>();
    CHECK(sizeof(bytesConstRef) == 16);
    {
        bytes in(128, 0);
        std::memcpy(in.data(), mh.data(), 32);
        in[63] = 27;
        std::memcpy(in.data() + 64, sig.data(), 64);
        auto ra = k1.recoverAddress(keccak, bytesConstRef(in));
        CHECK(!ra.first && ra.second.empty());
        in[63] = 29;
        CHECK(!k1.recoverAddress(keccak, bytesConstRef(in)).first);
        in[63] = 27;
        in[40] = 1;  // v = 27 + 2^k is not 27
        CHECK(!k1.recoverAddress(keccak, bytesConstRef(in)).first);
    }
    // v = 4 must throw InvalidSignature (SignatureTest.cpp:156-162); a wrong length too
    bytes bad = sig;
    bad[64] = 4;
    CHECK(throws_invalid([&] { k1.recover(mh, bytesConstRef(bad)); }));
    CHECK(throws_invalid([&] { k1.recover(mh, bytesConstRef(sig.data(), 64)); }));
    // a different hash recovers a different key (TxPoolTest.cpp:469-489): accepted
    HashType mh2 = hash_of("48bed44d1bcd124a28c27f343a817e5f5243190d3c52bf347daf876de1dbbf77");
    PublicPtr pub2 = k1.recover(mh2, bytesConstRef(sig));
    CHECK(pub2 && pub2->data() != pub->data());
    CHECK(!k1.verify(pub, mh2, bytesConstRef(sig)));
    // batch hook: entries of SignatureCrypto::recover, nullptr where it throws
    auto batch = secp.recoverBatch({mh, mh, mh2}, {bytesConstRef(sig), bytesConstRef(bad), bytesConstRef(sig)});
    CHECK(batch.size() == 3 && batch[0] && !batch[1] && batch[2]);
    CHECK(batch[0]->data() == pub->data() && batch[2]->data() == pub2->data());

    // SM2 KAT (SignatureTest.cpp:238-251): r || s || pub over SM3("abcd"), through m_verifier
    bytes sm2sig = unhex(
        "cd39bf939d999ca710576a629c962edfc28608701a3a7b61c971daeac5a1399c"
        "f4a7272fa80783e171c7fd5b038a3af4521f681ebe9fd44db3b60e750c438293"
        "f7dee65e76603ed7cd4c598d53cabe875c459e0fae4c6fd7b858189fd4741081"
        "e970bca0d5cb571a7ac30586aec71b23187d4b25e59143812f74a2744604d42b");
    HashType sm3abcd = hash_of("82ec580fe6d36ae4f81cae3c73f4a5b3b5a09c943172dc9053c69fd8e18dca1e");
    PublicPtr sp = s2.recover(sm3abcd, bytesConstRef(sm2sig));
    CHECK(sp && std::memcmp(sp->constData(), sm2sig.data() + 64, 64) == 0);
    CHECK(s2.verify(sp, sm3abcd, bytesConstRef(sm2sig)));
    bytes sm2bad = sm2sig;
    sm2bad[5] ^= 1;
    CHECK(throws_invalid([&] { s2.recover(sm3abcd, bytesConstRef(sm2bad)); }));
    CHECK(throws_invalid([&] { s2.recover(mh, bytesConstRef(sm2sig)); }));  // wrong hash: SM2 rejects
    auto sb = sm2.recoverBatch({sm3abcd, sm3abcd}, {bytesConstRef(sm2sig), bytesConstRef(sm2bad)});
    CHECK(sb.size() == 2 && sb[0] && !sb[1]);
    // the bytes overload (SM2Crypto.cpp:29-34) reaches the GPU through verify
    bytes sm2pub(sm2sig.begin() + 64, sm2sig.end());
    CHECK(s2.verify(std::make_shared<const bytes>(sm2pub), sm3abcd, bytesConstRef(sm2sig)));
    CHECK(!s2.verify(std::make_shared<const bytes>(sm2pub), sm3abcd, bytesConstRef(sm2bad)));
    {
        bytes in(160, 0);
        std::memcpy(in.data(), sm3abcd.data(), 32);
        std::memcpy(in.data() + 32, sm2pub.data(), 64);
        std::memcpy(in.data() + 96, sm2sig.data(), 64);
        // the reference's 16-byte copy (SM2Crypto.cpp:103): pub, r, s read as zero -> {false, {}} even for
        // the KAT's valid hash || pub || r || s
        auto ra = s2.recoverAddress(keccak, bytesConstRef(in));
        CHECK(!ra.first && ra.second.empty());
        in[100] ^= 1;
        CHECK(!s2.recoverAddress(keccak, bytesConstRef(in)).first);
    }
    // SM2 signature lengths (oracle/ec.c oracle_sm2_recover: only exactly 128 bytes recover).  The reference:
    // SM2Crypto::recover takes pub = every byte after r || s (SignatureDataWithPub.h:55-64); KeyImpl(64, pub)
    // throws InvalidKey below 64 bytes (KeyImpl.h:36-46) and keeps a longer one whole, which fast_sm2_verify's
    // hex2point("04" || pub) rejects (fast_sm2.cpp:142-160) -> InvalidSignature.  recoverBatch: nullptr for all.
    // verify with a KNOWN 64-byte key reads r || s only (SM2Crypto.cpp:71), so the length does not matter there.
    {
        bytes s127(sm2sig.begin(), sm2sig.begin() + 127);
        bytes s129 = sm2sig;
        s129.push_back(0);
        bytes s192 = sm2sig;
        s192.insert(s192.end(), 64, 0x11);
        bool invalidKey = false;
        try {
            s2.recover(sm3abcd, bytesConstRef(s127));
        } catch (const InvalidKey&) {
            invalidKey = true;
        }
        CHECK(invalidKey);
        CHECK(throws_invalid([&] { s2.recover(sm3abcd, bytesConstRef(s129)); }));
        CHECK(throws_invalid([&] { s2.recover(sm3abcd, bytesConstRef(s192)); }));
        CHECK(s2.verify(sp, sm3abcd, bytesConstRef(s127)));
        CHECK(s2.verify(sp, sm3abcd, bytesConstRef(s129)));
        CHECK(s2.verify(sp, sm3abcd, bytesConstRef(s192)));
        auto lb = sm2.recoverBatch({sm3abcd, sm3abcd, sm3abcd, sm3abcd},
            {bytesConstRef(sm2sig), bytesConstRef(s127), bytesConstRef(s129), bytesConstRef(s192)});
        CHECK(lb.size() == 4 && lb[0] && !lb[1] && !lb[2] && !lb[3]);
    }
    // a device SET in one process ({0, 0}: two shards on the one GPU here): batches sharded over it, single
    // calls taking its devices in turn -- same results
    {
        bcosgpu::ref::GpuSecp256k1Crypto secp2(std::vector<int>{0, 0});
        bcosgpu::ref::GpuSM2Crypto sm22(std::vector<int>{0, 0});
        std::vector<HashType> hs;
        std::vector<bytesConstRef> ss;
        for (int i = 0; i < 9; ++i) {
            hs.push_back(i % 3 == 2 ? mh2 : mh);
            ss.push_back(i % 3 == 1 ? bytesConstRef(bad) : bytesConstRef(sig));
        }
        auto b2 = secp2.recoverBatch(hs, ss);
        CHECK(b2.size() == 9);
        for (int i = 0; i < 9; ++i)
            CHECK(i % 3 == 1 ? !b2[i] : (b2[i] && b2[i]->data() == (i % 3 == 2 ? pub2 : pub)->data()));
        for (int i = 0; i < 4; ++i) CHECK(secp2.recover(mh, bytesConstRef(sig))->data() == pub->data());
        auto sb2 = sm22.recoverBatch({sm3abcd, sm3abcd, sm3abcd}, {bytesConstRef(sm2sig), bytesConstRef(sm2bad),
                                                                 bytesConstRef(sm2sig)});
        CHECK(sb2.size() == 3 && sb2[0] && !sb2[1] && sb2[2]);
        CHECK(secp2.devices().size() == 2 && sm22.device() == 0);
    }
    // SM2 recoverAddress with an engine failure throws SignException (not {false, {}})
    {
        bcosgpu::ref::GpuSM2Crypto badSm2(64);
        bytes in(160, 0);
        std::memcpy(in.data(), sm3abcd.data(), 32);
        std::memcpy(in.data() + 32, sm2pub.data(), 64);
        std::memcpy(in.data() + 96, sm2sig.data(), 64);
        CHECK(throws_sign_exception([&] { badSm2.recoverAddress(keccak, bytesConstRef(in)); }));
        // shorter input is zero-padded: no key, no address
        CHECK(!s2.recoverAddress(keccak, bytesConstRef(in.data(), 100)).first);
    }

    // the wedpr-shaped m_verifier: WEDPR_SUCCESS / WEDPR_ERROR
    SM2Probe probe(0);
    CHECK(probe.callVerifier(sm2pub, sm3abcd, sm2sig) == WEDPR_SUCCESS);
    CHECK(probe.callVerifier(sm2pub, sm3abcd, sm2bad) == WEDPR_ERROR);

    // calls from another thread run on the object's device without any per-thread setup
    {
        bool okThread = false;
        std::thread t([&] { okThread = k1.recover(mh, bytesConstRef(sig))->data() == pub->data() &&
                                       s2.recover(sm3abcd, bytesConstRef(sm2sig)) != nullptr; });
        t.join();
        CHECK(okThread);
    }

    // injected engine failure (a device index the engine rejects): SignException on both suites, from
    // every entry point, never InvalidSignature (TxValidator.cpp:54-61 would reject the tx); the
    // wedpr-shaped verifier returns BCOSGPU_WEDPR_ENGINE_ERROR
    {
        bcosgpu::ref::GpuSecp256k1Crypto badK1(64);
        bcosgpu::ref::GpuSM2Crypto badSm2(64);
        SignatureCrypto& bk = badK1;
        SignatureCrypto& bs = badSm2;
        CHECK(throws_sign_exception([&] { bk.recover(mh, bytesConstRef(sig)); }));
        CHECK(throws_sign_exception([&] { bk.verify(pub, mh, bytesConstRef(sig)); }));
        CHECK(throws_sign_exception([&] { bk.verify(std::make_shared<const bytes>(pub->data()), mh, bytesConstRef(sig)); }));
        CHECK(throws_sign_exception([&] { badK1.recoverBatch({mh}, {bytesConstRef(sig)}); }));
        CHECK(throws_sign_exception([&] { bs.recover(sm3abcd, bytesConstRef(sm2sig)); }));
        CHECK(throws_sign_exception([&] { bs.verify(sp, sm3abcd, bytesConstRef(sm2sig)); }));
        CHECK(throws_sign_exception([&] { badSm2.recoverBatch({sm3abcd}, {bytesConstRef(sm2sig)}); }));
        SM2Probe badProbe(64);
        CHECK(badProbe.callVerifier(sm2pub, sm3abcd, sm2sig) == BCOSGPU_WEDPR_ENGINE_ERROR);
        uint8_t out64[64];
        CHECK(bcosgpu_secp256k1_recover(64, mh.data(), sig.data(), 65, out64) < 0);
    }

    printf(fails ? "sigcrypto_test: %d failures\n" : "sigcrypto_test: ok\n", fails);
    return fails ? 1 : 0;
}
