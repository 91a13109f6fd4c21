/*
 * bcos_gpu_crypto.hpp -- drop-in bcos::crypto::SignatureCrypto implementations over libbcosgpu.so,
 * meant to be compiled INSIDE the reference tree (its bcos-crypto headers, wedpr-crypto, Boost).
 *
 *   GpuSecp256k1Crypto : bcos::crypto::Secp256k1Crypto        (Secp256k1Crypto.h:37-72)
 *       recover (Secp256k1Crypto.cpp:79-93) and verify (:51-63) run on the GPU through the C ABI;
 *       sign / key generation stay on the host (wedpr), as signing must be constant-time.
 *   GpuSM2Crypto : bcos::crypto::SM2Crypto                    (SM2Crypto.h:31-67)
 *       m_verifier = bcosgpu_wedpr_sm2_verify, so SM2Crypto::verify and ::recover
 *       (SM2Crypto.cpp:66-92) run on the GPU unchanged; m_signer stays wedpr's.
 *   recoverBatch(hashes, signatures) on both: one device call for a whole batch -- the hook the
 *       batch sites (TransactionSync::importDownloadedTxs' parallel_for, TransactionSync.cpp:516-548)
 *       are rewired to; entry i is the recovered key or nullptr where SignatureCrypto::recover would
 *       throw InvalidSignature.
 *
 * Failures throw what the reference throws: InvalidSignature via BOOST_THROW_EXCEPTION with an
 * errinfo_comment (Secp256k1Crypto.cpp:86-91, SM2Crypto.cpp:89-91); an engine error (no gfx950 device,
 * HIP failure) throws bcos::crypto::SignException with the engine's message.  Selection in
 * ProtocolInitializer::createCryptoSuite (libinitializer/ProtocolInitializer.cpp:102-124) is the only
 * other line to change: INTEGRATION.md §2.  tests/cpp/sigcrypto_test.cpp compiles this header against
 * a mirror of those interfaces (tests/cpp/mirror/) and runs the reference KATs through it.
 */
#pragma once
#include <bcos-crypto/interfaces/crypto/Signature.h>
#include <bcos-crypto/signature/Exceptions.h>
#include <bcos-crypto/signature/key/KeyImpl.h>
#include <bcos-crypto/signature/secp256k1/Secp256k1Crypto.h>
#include <bcos-crypto/signature/secp256k1/Secp256k1KeyPair.h>
#include <bcos-crypto/signature/sm2/SM2Crypto.h>
#include <bcos-crypto/signature/sm2/SM2KeyPair.h>
#include <wedpr-crypto/WedprCrypto.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "bcos_gpu_wedpr.h"

namespace bcosgpu
{
namespace ref
{
inline void initDevice(int device)
{
    if (bcosgpu_init(device) != BCOSGPU_OK)
    {
        BOOST_THROW_EXCEPTION(bcos::crypto::SignException() << bcos::errinfo_comment(
                                  std::string("bcosgpu_init: ") + bcosgpu_last_error()));
    }
}

inline void engineCheck(int rc, const char* what)
{
    if (rc != BCOSGPU_OK)
    {
        BOOST_THROW_EXCEPTION(bcos::crypto::SignException() << bcos::errinfo_comment(
                                  std::string(what) + ": " + bcosgpu_last_error()));
    }
}

class GpuSecp256k1Crypto : public bcos::crypto::Secp256k1Crypto
{
public:
    using Ptr = std::shared_ptr<GpuSecp256k1Crypto>;
    explicit GpuSecp256k1Crypto(int _device = 0) { initDevice(_device); }
    ~GpuSecp256k1Crypto() override = default;

    // Secp256k1Crypto::recover -> secp256k1Recover (Secp256k1Crypto.cpp:79-93)
    bcos::crypto::PublicPtr recover(
        const bcos::crypto::HashType& _hash, bcos::bytesConstRef _signatureData) const override
    {
        auto pub = std::make_shared<bcos::crypto::KeyImpl>(bcos::crypto::SECP256K1_PUBLIC_LEN);
        uint8_t ok = 0;
        if (_signatureData.size() == (size_t)bcos::crypto::SECP256K1_SIGNATURE_LEN)
        {
            engineCheck(bcosgpu_secp256k1_recover_batch(_hash.data(), _signatureData.data(), 1,
                            (uint8_t*)pub->mutableData(), nullptr, &ok),
                "bcosgpu_secp256k1_recover_batch");
        }
        if (!ok)
        {
            BOOST_THROW_EXCEPTION(bcos::crypto::InvalidSignature() << bcos::errinfo_comment(
                                      "invalid signature: secp256k1Recover failed, msgHash : " +
                                      _hash.hex()));
        }
        return pub;
    }

    // Secp256k1Crypto::verify -> secp256k1Verify (Secp256k1Crypto.cpp:51-63): libsecp256k1 verify
    // semantics (low-S), only r || s read
    bool verify(bcos::crypto::PublicPtr _pubKey, const bcos::crypto::HashType& _hash,
        bcos::bytesConstRef _signatureData) const override
    {
        if (!_pubKey || _pubKey->size() != (size_t)bcos::crypto::SECP256K1_PUBLIC_LEN ||
            _signatureData.size() < 64)
        {
            return false;
        }
        uint8_t ok = 0;
        engineCheck(bcosgpu_verify_batch(BCOSGPU_SUITE_SECP256K1, (const uint8_t*)_pubKey->constData(),
                        _hash.data(), _signatureData.data(), 64, 1, &ok),
            "bcosgpu_verify_batch");
        return ok != 0;
    }
    using bcos::crypto::Secp256k1Crypto::verify;

    // batch hook: recover every signature of a batch in one device call
    std::vector<bcos::crypto::PublicPtr> recoverBatch(const std::vector<bcos::crypto::HashType>& _hashes,
        const std::vector<bcos::bytesConstRef>& _signatures) const
    {
        const size_t n = _hashes.size();
        std::vector<bcos::crypto::PublicPtr> out(n);
        if (n == 0 || _signatures.size() != n)
        {
            return out;
        }
        std::vector<uint8_t> h(32 * n), s(65 * n, 0), pub(64 * n), ok(n, 0);
        std::vector<bool> wellFormed(n);
        for (size_t i = 0; i < n; ++i)
        {
            std::memcpy(h.data() + 32 * i, _hashes[i].data(), 32);
            wellFormed[i] = _signatures[i].size() == (size_t)bcos::crypto::SECP256K1_SIGNATURE_LEN;
            if (wellFormed[i])
            {
                std::memcpy(s.data() + 65 * i, _signatures[i].data(), 65);
            }
        }
        engineCheck(
            bcosgpu_secp256k1_recover_batch(h.data(), s.data(), n, pub.data(), nullptr, ok.data()),
            "bcosgpu_secp256k1_recover_batch");
        for (size_t i = 0; i < n; ++i)
        {
            if (ok[i] && wellFormed[i])
            {
                auto key = std::make_shared<bcos::crypto::KeyImpl>(bcos::crypto::SECP256K1_PUBLIC_LEN);
                std::memcpy(key->mutableData(), pub.data() + 64 * i, 64);
                out[i] = key;
            }
        }
        return out;
    }
};

class GpuSM2Crypto : public bcos::crypto::SM2Crypto
{
public:
    using Ptr = std::shared_ptr<GpuSM2Crypto>;
    explicit GpuSM2Crypto(int _device = 0)
    {
        initDevice(_device);
        m_verifier = bcosgpu_wedpr_sm2_verify;  // SM2Crypto.h:64-65: verify and recover on the GPU
    }
    ~GpuSM2Crypto() override = default;

    // batch hook: SM2Crypto::recover (verify against the embedded key) for a whole batch
    std::vector<bcos::crypto::PublicPtr> recoverBatch(const std::vector<bcos::crypto::HashType>& _hashes,
        const std::vector<bcos::bytesConstRef>& _signatures) const
    {
        const size_t n = _hashes.size();
        std::vector<bcos::crypto::PublicPtr> out(n);
        if (n == 0 || _signatures.size() != n)
        {
            return out;
        }
        std::vector<uint8_t> h(32 * n), s(128 * n, 0), ok(n, 0);
        std::vector<bool> wellFormed(n);
        for (size_t i = 0; i < n; ++i)
        {
            std::memcpy(h.data() + 32 * i, _hashes[i].data(), 32);
            // SignatureDataWithPub needs r || s || pub (128 B); SM2Crypto::recover reads pub from it
            wellFormed[i] = _signatures[i].size() >= 128;
            if (wellFormed[i])
            {
                std::memcpy(s.data() + 128 * i, _signatures[i].data(), 128);
            }
        }
        engineCheck(bcosgpu_sm2_verify_batch(h.data(), s.data(), n, nullptr, ok.data()),
            "bcosgpu_sm2_verify_batch");
        for (size_t i = 0; i < n; ++i)
        {
            if (ok[i] && wellFormed[i])
            {
                auto key = std::make_shared<bcos::crypto::KeyImpl>(bcos::crypto::SM2_PUBLIC_KEY_LEN);
                std::memcpy(key->mutableData(), _signatures[i].data() + 64, 64);
                out[i] = key;
            }
        }
        return out;
    }
};
}  // namespace ref
}  // namespace bcosgpu
