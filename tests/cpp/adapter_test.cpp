// adapter_test.cpp -- C++ parity test through include/bcos_gpu.hpp (the reference-shaped adapters),
// written like bcos-crypto/test/unittests/{HashTest,SignatureTest}.cpp.  Exit 0 = pass, 77 = no GPU.
#include <cstdio>
#include <cstring>
#include <string>
#include "../../include/bcos_gpu.hpp"

using namespace bcosgpu;

static std::string hex(const uint8_t* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}
static bytes unhex(const char* h) {
    bytes b(strlen(h) / 2);
    for (size_t i = 0; i < b.size(); ++i) sscanf(h + 2 * i, "%2hhx", &b[i]);
    return b;
}
static int fails = 0;
#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

int main() {
    if (bcosgpu_device_count() <= 0 || bcosgpu_init(0) != 0) {
        printf("no gfx950 device: %s\n", bcosgpu_last_error());
        return 77;
    }
    GpuKeccak256 k;
    GpuSM3 sm3;
    auto h = [](const char* s) { return bytes(s, s + strlen(s)); };
    // HashTest.cpp:59-99
    CHECK(hex(k.hash(h("")).data(), 32) == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470");
    CHECK(hex(k.hash(h("abcde")).data(), 32) == "6377c7e66081cb65e473c1b95db5195a27d04a7108b468890224bedbe1a8a6eb");
    CHECK(hex(sm3.hash(h("hello")).data(), 32) == "becbbfaae6548b8bf0cfcad5a27183cd1be6093b1cceccc303d9c61d0a645268");
    // ecrecover vector (EVMPrecompiledTest.cpp:58-72)
    HashType mh{};
    bytes hb = unhex("38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e");
    std::memcpy(mh.data(), hb.data(), 32);
    bytes sig = hb;
    bytes s = unhex("789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02");
    sig.insert(sig.end(), s.begin(), s.end());
    sig.push_back(0);
    GpuSecp256k1Crypto secp;
    bytes pub = secp.recover(mh, sig.data(), sig.size());
    CHECK(hex(right160(k.hash(pub)).data(), 20) == "ceaccac640adf55b2028469bd36ba501f28b699d");
    CHECK(secp.verify(pub.data(), mh, sig.data(), sig.size()));  // Secp256k1Crypto::verify, known key
    {   // EVM ecRecover precompile input hash || v=27 || r || s (EVMPrecompiledTest.cpp:58-72)
        bytes in(128, 0);
        std::memcpy(in.data(), hb.data(), 32);
        in[63] = 27;
        std::memcpy(in.data() + 64, hb.data(), 32);
        std::memcpy(in.data() + 96, s.data(), 32);
        auto r = ecRecover(in.data(), in.size());
        CHECK(r.first && r.second.size() == 32);
        CHECK(hex(r.second.data(), 32) == "000000000000000000000000ceaccac640adf55b2028469bd36ba501f28b699d");
        in[63] = 29;
        r = ecRecover(in.data(), in.size());
        CHECK(r.first && r.second.empty());
    }
    sig[64] = 4;  // SignatureTest.cpp:156-162
    bool threw = false;
    try { secp.recover(mh, sig.data(), sig.size()); } catch (const InvalidSignature&) { threw = true; }
    CHECK(threw);
    // SM2 KAT (SignatureTest.cpp:238-251)
    HashType sh = sm3.hash(h("abcd"));
    bytes s2 = unhex("cd39bf939d999ca710576a629c962edfc28608701a3a7b61c971daeac5a1399cf4a7272fa80783e171c7fd5b038a3af4521f681ebe9fd44db3b60e750c438293f7dee65e76603ed7cd4c598d53cabe875c459e0fae4c6fd7b858189fd4741081e970bca0d5cb571a7ac30586aec71b23187d4b25e59143812f74a2744604d42b");
    GpuSM2Crypto sm2;
    CHECK(sm2.recover(sh, s2.data(), s2.size()) == bytes(s2.begin() + 64, s2.end()));
    CHECK(sm2.verify(s2.data() + 64, sh, s2.data(), 64));
    s2[3] ^= 1;
    threw = false;
    try { sm2.recover(sh, s2.data(), s2.size()); } catch (const InvalidSignature&) { threw = true; }
    CHECK(threw);
    // Merkle<SM3,16> over merkleBench leaves, n = 17 (reference root)
    std::vector<HashType> leaves;
    for (uint64_t i = 0; i < 17; ++i) leaves.push_back(sm3.hash(reinterpret_cast<const uint8_t*>(&i), 8));
    std::vector<HashType> out;
    GpuMerkle<BCOSGPU_SM3, 16>().generateMerkle(leaves, out);
    CHECK(out.size() == 5);
    CHECK(hex(out.back().data(), 32) == "1f9ac75f82e1f0b6955634b2fc48b08ab48518d8e6716151c12345d73f6cecfe");
    threw = false;
    try { GpuMerkle<BCOSGPU_SM3, 16>().generateMerkle({}, out); } catch (const std::invalid_argument&) { threw = true; }
    CHECK(threw);
    // the same tree as merkleBench stores it (vector<bytes>, merkleBench.cpp:53-56): 4-byte count records
    std::vector<std::vector<char>> vb;
    GpuMerkle<BCOSGPU_SM3, 16>().generateMerkle(leaves, vb);
    CHECK(vb.size() == out.size());
    for (size_t i = 0; i < vb.size() && i < out.size(); ++i) {
        const bool record = i == 0 || i == 3;  // [count 2][2 nodes][count 1][root]
        CHECK(vb[i].size() == (record ? 4u : 32u));
        CHECK(std::memcmp(vb[i].data(), out[i].data(), vb[i].size()) == 0);
    }
    std::vector<bytes> one;
    GpuMerkle<BCOSGPU_KECCAK256, 2>().generateMerkle({leaves[0]}, one);
    CHECK(one.size() == 1 && one[0].size() == 32 && std::memcmp(one[0].data(), leaves[0].data(), 32) == 0);
    // Merkle proofs (testMerkle.cpp:91-121): every leaf verifies, a zero hash does not, empty proof throws
    GpuMerkle<BCOSGPU_SM3, 16> m16;
    for (uint64_t i = 0; i < leaves.size(); ++i) {
        std::vector<HashType> proof;
        m16.generateMerkleProof(leaves, i, proof);
        CHECK(m16.verifyMerkleProof(proof, leaves[i], out.back()));
        CHECK(!m16.verifyMerkleProof(proof, HashType{}, out.back()));
    }
    threw = false;
    try { m16.verifyMerkleProof({}, leaves[0], out.back()); } catch (const std::invalid_argument&) { threw = true; }
    CHECK(threw);
    // calculateTransactionRoot over a batch of blocks: Keccak width 2, n = 17 and an empty block
    auto roots = calculateRoots<BCOSGPU_KECCAK256>({leaves, {}});
    CHECK(roots.size() == 2);
    CHECK(hex(roots[0].data(), 32) == "741f553a7d060d82679d4dd31c12fc647d3871226808312d8807ace6d4ac5b50");
    CHECK(roots[1] == HashType{});
    printf(fails ? "adapter_test: %d failures\n" : "adapter_test: ok\n", fails);
    return fails ? 1 : 0;
}
