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
#include <algorithm>
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
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
    /* Secp256k1Crypto::verify -> secp256k1Verify (Secp256k1Crypto.cpp:51-63): r || s = sig[0:64] */
    bool verify(const uint8_t pub[64], const HashType& hash, const uint8_t* sig, size_t sig_len) const {
        if (sig_len < 64) return false;
        uint8_t ok = 0;
        check(bcosgpu_verify_batch(BCOSGPU_SUITE_SECP256K1, pub, hash.data(), sig, 64, 1, &ok));
        return ok != 0;
    }
    /* batch verify with known keys (sealer signatures): item i = pubs + 64 i, hashes + 32 i, sigs + stride i */
    void verify_batch(const uint8_t* pubs, const uint8_t* hashes, const uint8_t* sigs, size_t stride, size_t n,
                      uint8_t* ok) const {
        check(bcosgpu_verify_batch(BCOSGPU_SUITE_SECP256K1, pubs, hashes, sigs, stride, n, ok));
    }
};

class GpuSM2Crypto {
public:
    static constexpr size_t SIGNATURE_LEN = 64; /* SM2_SIGNATURE_LEN: r || s */
    /* SM2Crypto::verify (SM2Crypto.cpp:66-79): only sig[0:64] is used */
    bool verify(const uint8_t pub[64], const HashType& hash, const uint8_t* sig, size_t sig_len) const {
        if (sig_len < SIGNATURE_LEN) return false;
        uint8_t ok = 0;
        check(bcosgpu_verify_batch(BCOSGPU_SUITE_SM2, pub, hash.data(), sig, SIGNATURE_LEN, 1, &ok));
        return ok != 0;
    }
    void verify_batch(const uint8_t* pubs, const uint8_t* hashes, const uint8_t* sigs, size_t stride, size_t n,
                      uint8_t* ok) const {
        check(bcosgpu_verify_batch(BCOSGPU_SUITE_SM2, pubs, hashes, sigs, stride, n, ok));
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
    /* generateMerkle into a vector of byte buffers -- BlockImpl's m_inner->transactionsMerkle
     * (vector<vector<char>>, BlockImpl.h:136) and merkleBench's vector<bytes> (merkleBench.cpp:53-56):
     * count records are 4-byte entries (Merkle.h:213-217 resizeTo(output, 4)), nodes 32 bytes.
     * Bytes = any resizable byte container (std::vector<char>, std::vector<uint8_t>, bcos::bytes). */
    template <class Bytes>
    void generateMerkle(const std::vector<HashType>& originHashes, std::vector<Bytes>& out) const {
        if (originHashes.empty()) throw std::invalid_argument("Empty input");
        const size_t n = originHashes.size();
        std::vector<uint8_t> flat(bcosgpu_merkle_bytes_size(n, static_cast<int>(width)));
        HashType root{};
        check(bcosgpu_merkle_root(HASHER, static_cast<int>(width), BCOSGPU_MERKLE_NEW_BYTES, originHashes[0].data(), n,
                                  root.data(), flat.data()));
        out.clear();
        auto put = [&out](const uint8_t* p, size_t len) {
            out.emplace_back(len);
            std::copy(p, p + len, reinterpret_cast<uint8_t*>(&out.back()[0]));
        };
        if (n == 1) {
            put(flat.data(), 32);
            return;
        }
        for (size_t at = 0; at < flat.size();) {
            const uint32_t cnt = (uint32_t(flat[at]) << 24) | (uint32_t(flat[at + 1]) << 16) |
                                 (uint32_t(flat[at + 2]) << 8) | uint32_t(flat[at + 3]);
            put(flat.data() + at, 4);
            at += 4;
            for (uint32_t k = 0; k < cnt; ++k, at += 32) put(flat.data() + at, 32);
        }
    }
    /* generateMerkleProof(originHashes, index, out) (Merkle.h:121-168): out is replaced (the reference
     * appends to a caller-cleared vector); index out of range throws std::invalid_argument */
    void generateMerkleProof(const std::vector<HashType>& originHashes, uint64_t index, std::vector<HashType>& out) const {
        if (originHashes.empty()) throw std::invalid_argument("Empty input");
        if (index >= originHashes.size()) throw std::invalid_argument("Out of range!");
        out.resize(bcosgpu_merkle_proof_stride(originHashes.size(), static_cast<int>(width)));
        uint32_t len = 0;
        check(bcosgpu_merkle_proofs(HASHER, static_cast<int>(width), originHashes[0].data(), originHashes.size(), &index,
                                    1, out[0].data(), &len));
        out.resize(len);
    }
    /* verifyMerkleProof(proof, hash, root) (Merkle.h:45-81); an empty proof throws std::invalid_argument */
    bool verifyMerkleProof(const std::vector<HashType>& proof, const HashType& hash, const HashType& root) const {
        if (proof.empty()) throw std::invalid_argument("Empty input proof!");
        const uint32_t len = static_cast<uint32_t>(proof.size());
        uint8_t ok = 0;
        check(bcosgpu_merkle_verify_proofs(HASHER, proof[0].data(), proof.size(), &len, hash.data(), root.data(), 0, 1, &ok));
        return ok == 1;
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

/* calculateTransactionRoot / calculateReceiptRoot of many blocks in one engine call; an empty block
 * gives the zero hash (BlockImpl.h:114-119, :159-163). */
template <int HASHER>
inline std::vector<HashType> calculateRoots(const std::vector<std::vector<HashType>>& blocks) {
    std::vector<uint64_t> off(blocks.size() + 1, 0);
    std::vector<HashType> leaves;
    for (size_t b = 0; b < blocks.size(); ++b) {
        leaves.insert(leaves.end(), blocks[b].begin(), blocks[b].end());
        off[b + 1] = leaves.size();
    }
    std::vector<HashType> roots(blocks.size());
    if (blocks.empty()) return roots;
    static const HashType zero{};
    check(bcosgpu_merkle_roots_batch(HASHER, 2, leaves.empty() ? zero.data() : leaves[0].data(), off.data(),
                                     blocks.size(), roots[0].data()));
    return roots;
}

/* BlockImpl::calculateReceiptRoot (BlockImpl.h:156-183) for many blocks in one engine call: every receipt
 * hashed on the GPU (impl_calculate<Hasher>(TransactionReceipt), TarsHashable.h:43-75, a set dataHash
 * used as is), then each block's width-2 root; a block without receipts gives the zero hash.
 * receiptHashes (nullable) receives every receipt's hash, blocks back to back. */
template <int HASHER>
inline std::vector<HashType> calculateReceiptRoots(const std::vector<std::vector<bcosgpu_TransactionReceiptData>>& blocks,
                                                   std::vector<HashType>* receiptHashes = nullptr) {
    std::vector<uint64_t> off(blocks.size() + 1, 0);
    std::vector<bcosgpu_TransactionReceiptData> all;
    for (size_t b = 0; b < blocks.size(); ++b) {
        all.insert(all.end(), blocks[b].begin(), blocks[b].end());
        off[b + 1] = all.size();
    }
    std::vector<HashType> roots(blocks.size());
    if (receiptHashes) receiptHashes->assign(all.size(), HashType{});
    if (blocks.empty()) return roots;
    check(bcosgpu_receipt_roots(HASHER, all.data(), off.data(), blocks.size(), roots[0].data(),
                                receiptHashes && !all.empty() ? (*receiptHashes)[0].data() : nullptr));
    return roots;
}

/* BlockImpl::calculateReceiptRoot for one block */
template <int HASHER>
inline HashType calculateReceiptRoot(const std::vector<bcosgpu_TransactionReceiptData>& receipts) {
    return calculateReceiptRoots<HASHER>({receipts})[0];
}

/* EVM ecRecover precompile (bcos-executor/src/vm/Precompiled.cpp:443-482): {true, 32-byte output}
 * on success, {true, {}} on failure; `in` is read as 128 zero-padded bytes. */
inline std::pair<bool, bytes> ecRecover(const uint8_t* in, size_t len) {
    alignas(16) uint8_t buf[128] = {0};
    for (size_t i = 0; i < len && i < 128; ++i) buf[i] = in[i];
    uint8_t out[32], ok = 0;
    check(bcosgpu_ecrecover_batch(buf, 1, out, &ok));
    if (!ok) return {true, bytes()};
    return {true, bytes(out, out + 32)};
}

}  // namespace bcosgpu
#endif
