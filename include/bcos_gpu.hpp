/*
 * bcos_gpu.hpp -- header-only C++ adapters over the C ABI (bcos_gpu.h) with the shapes of the
 * reference's interfaces, so that the reference's call sites can be rewired without other changes:
 *
 *   bcos::crypto::Hash::hash(bytesConstRef) -> h256            interfaces/crypto/Hash.h:44
 *       -> bcosgpu::GpuKeccak256 / GpuSM3 ::hash, plus batch hash_batch()
 *   bcos::crypto::SignatureCrypto::recover(HashType, bytesConstRef) -> PublicPtr (throws InvalidSignature)
 *                                                              interfaces/crypto/Signature.h:53-54
 *       -> bcosgpu::GpuSecp256k1Crypto / GpuSM2Crypto ::recover, plus recover_batch()
 *   SignatureCrypto::verify(PublicPtr, HashType, bytesConstRef) -> bool       Signature.h:45-48
 *   bcos::crypto::merkle::Merkle<Hasher, width>::generateMerkle(originHashes, out)  merkle/Merkle.h:170-208
 *       -> bcosgpu::GpuMerkle<width>::generateMerkle (same output vector layout)
 *
 * The reference's own types (bcos::bytes, h256, KeyImpl, ...) are not available here; these adapters
 * use std::vector<uint8_t> / std::array, and INTEGRATION.md shows the few lines that wrap them into a
 * bcos::crypto::SignatureCrypto subclass.  Errors from the engine throw std::runtime_error; crypto
 * failures throw bcosgpu::InvalidSignature exactly where the reference throws InvalidSignature.
 */
#ifndef BCOS_GPU_HPP
#define BCOS_GPU_HPP
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "bcos_gpu.h"

namespace bcosgpu {

using bytes = std::vector<uint8_t>;
using HashType = std::array<uint8_t, 32>;

struct InvalidSignature : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void check(int rc) {
    if (rc != BCOSGPU_OK) throw std::runtime_error(std::string("bcosgpu: ") + bcosgpu_last_error());
}

// ---------------------------------------------------------------- Hash
template <int HASHER>
class GpuHash {
public:
    HashType hash(const uint8_t* data, size_t len) const {
        uint64_t off[2] = {0, len};
        HashType out{};
        check(bcosgpu_hash_batch(HASHER, len ? data : &zero_, off, 1, out.data()));
        return out;
    }
    HashType hash(const bytes& b) const { return hash(b.data(), b.size()); }
    /* batch: message i = data[offsets[i] .. offsets[i+1]) */
    std::vector<HashType> hash_batch(const bytes& data, const std::vector<uint64_t>& offsets) const {
        const size_t n = offsets.empty() ? 0 : offsets.size() - 1;
        std::vector<HashType> out(n);
        if (n) check(bcosgpu_hash_batch(HASHER, data.empty() ? &zero_ : data.data(), offsets.data(), n, out[0].data()));
        return out;
    }

private:
    static constexpr uint8_t zero_ = 0;
};
using GpuKeccak256 = GpuHash<BCOSGPU_KECCAK256>;
using GpuSM3 = GpuHash<BCOSGPU_SM3>;

inline std::array<uint8_t, 20> right160(const HashType& h) {
    std::array<uint8_t, 20> a{};
    for (int i = 0; i < 20; ++i) a[i] = h[12 + i];
    return a;
}

// ---------------------------------------------------------------- SignatureCrypto
class GpuSecp256k1Crypto {
public:
    static constexpr size_t SIGNATURE_LEN = 65; /* SECP256K1_SIGNATURE_LEN (Secp256k1Crypto.h:29) */
    /* Secp256k1Crypto::recover (Secp256k1Crypto.h:57-60): 64-byte public key or InvalidSignature */
    bytes recover(const HashType& hash, const uint8_t* sig, size_t sig_len) const {
        if (sig_len != SIGNATURE_LEN) throw InvalidSignature("invalid signature: secp256k1Recover failed");
        bytes pub(64);
        uint8_t ok = 0;
        check(bcosgpu_secp256k1_recover_batch(hash.data(), sig, 1, pub.data(), nullptr, &ok));
        if (!ok) throw InvalidSignature("invalid signature: secp256k1Recover failed");
        return pub;
    }
    /* batch recover: hashes n x 32, sigs n x 65 -> pubs n x 64, addrs n x 20 (keccak), ok[n] */
    void recover_batch(const uint8_t* hashes, const uint8_t* sigs, size_t n, uint8_t* pubs, uint8_t* addrs,
                       uint8_t* ok) const {
        check(bcosgpu_secp256k1_recover_batch(hashes, sigs, n, pubs, addrs, ok));
    }
};

class GpuSM2Crypto {
public:
    static constexpr size_t SIGNATURE_LEN = 64; /* SM2_SIGNATURE_LEN: r || s */
    /* SM2Crypto::verify (SM2Crypto.cpp:66-79): only sig[0:64] is used */
    bool verify(const uint8_t pub[64], const HashType& hash, const uint8_t* sig, size_t sig_len) const {
        if (sig_len < SIGNATURE_LEN) return false;
        uint8_t s[128], ok = 0;
        for (int i = 0; i < 64; ++i) { s[i] = sig[i]; s[64 + i] = pub[i]; }
        check(bcosgpu_sm2_verify_batch(hash.data(), s, 1, nullptr, &ok));
        return ok != 0;
    }
    /* SM2Crypto::recover (SM2Crypto.cpp:81-92): verify with the embedded key, return it */
    bytes recover(const HashType& hash, const uint8_t* sig, size_t sig_len) const {
        if (sig_len != 128) throw InvalidSignature("invalid signature: sm2 recover public key failed");
        uint8_t ok = 0;
        check(bcosgpu_sm2_verify_batch(hash.data(), sig, 1, nullptr, &ok));
        if (!ok) throw InvalidSignature("invalid signature: sm2 recover public key failed");
        return bytes(sig + 64, sig + 128);
    }
    void recover_batch(const uint8_t* hashes, const uint8_t* sigs128, size_t n, uint8_t* addrs, uint8_t* ok) const {
        check(bcosgpu_sm2_verify_batch(hashes, sigs128, n, addrs, ok));
    }
};

// ---------------------------------------------------------------- Merkle
template <int HASHER, size_t width = 2>
class GpuMerkle {
    static_assert(width >= 2, "Width too short, at least 2");

public:
    /* generateMerkle (Merkle.h:170-208): out = the reference's output vector (count records are
     * 32-byte entries with the big-endian count in bytes 0..3, as in Merkle<..>'s std::array case) */
    void generateMerkle(const std::vector<HashType>& originHashes, std::vector<HashType>& out) const {
        if (originHashes.empty()) throw std::invalid_argument("Empty input");
        out.resize(bcosgpu_merkle_size(originHashes.size(), static_cast<int>(width)));
        HashType root{};
        check(bcosgpu_merkle_root(HASHER, static_cast<int>(width), BCOSGPU_MERKLE_NEW, originHashes[0].data(),
                                  originHashes.size(), root.data(), out[0].data()));
    }
    HashType root(const std::vector<HashType>& originHashes) const {
        if (originHashes.empty()) throw std::invalid_argument("Empty input");
        HashType r{};
        check(bcosgpu_merkle_root(HASHER, static_cast<int>(width), BCOSGPU_MERKLE_NEW, originHashes[0].data(),
                                  originHashes.size(), r.data(), nullptr));
        return r;
    }
};

/* BlockImpl::calculateTransactionRoot (BlockImpl.h:111-154): width-2 root, zero hash when empty */
template <int HASHER>
inline HashType calculateTransactionRoot(const std::vector<HashType>& txHashes) {
    if (txHashes.empty()) return HashType{};
    return GpuMerkle<HASHER, 2>().root(txHashes);
}

}  // namespace bcosgpu
#endif
