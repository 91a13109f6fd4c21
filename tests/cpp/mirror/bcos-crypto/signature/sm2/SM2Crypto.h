// mirror of the SM2Crypto class shape (test infrastructure, ../../../README.md): verify / recover
// go through m_verifier as SM2Crypto.cpp:66-92 does; the host-side members only throw
#pragma once
#include <bcos-crypto/signature/Exceptions.h>
#include <bcos-crypto/signature/key/KeyImpl.h>
#include <bcos-crypto/signature/sm2/SM2KeyPair.h>
#include <wedpr-crypto/WedprCrypto.h>
#include <algorithm>
#include <functional>
namespace bcos
{
namespace crypto
{
const int SM2_SIGNATURE_LEN = 64;
class SM2Crypto : public SignatureCrypto
{
public:
    SM2Crypto() = default;
    ~SM2Crypto() override = default;
    std::shared_ptr<bytes> sign(const KeyPairInterface&, const HashType&, bool) const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
    bool verify(PublicPtr _pubKey, const HashType& _hash, bytesConstRef _signatureData) const override
    {
        CInputBuffer publicKey{_pubKey->constData(), _pubKey->size()};
        CInputBuffer messageHash{(const char*)_hash.data(), HashType::SIZE};
        CInputBuffer signature{(const char*)_signatureData.data(), SM2_SIGNATURE_LEN};
        return m_verifier(&publicKey, &messageHash, &signature) == WEDPR_SUCCESS;
    }
    bool verify(std::shared_ptr<const bytes> _pubKeyBytes, const HashType& _hash,
        bytesConstRef _signatureData) const override
    {
        return verify(std::make_shared<KeyImpl>(64, _pubKeyBytes), _hash, _signatureData);
    }
    // SM2Crypto.cpp:81-92: pub = every byte after r || s (SignatureDataWithPub::decode,
    // SignatureDataWithPub.h:55-64), KeyImpl(64, pub) throws InvalidKey when shorter than 64
    // (KeyImpl.h:36-46) and keeps all of them otherwise; then the virtual verify
    PublicPtr recover(const HashType& _hash, bytesConstRef _signData) const override
    {
        auto pubBytes = std::make_shared<bytes>();
        if (_signData.size() > (size_t)SM2_SIGNATURE_LEN)
        {
            pubBytes->assign(_signData.data() + SM2_SIGNATURE_LEN, _signData.data() + _signData.size());
        }
        auto pub = std::make_shared<KeyImpl>(64, pubBytes);
        if (verify(pub, _hash, _signData))
        {
            return pub;
        }
        BOOST_THROW_EXCEPTION(InvalidSignature() << errinfo_comment(
                                  "invalid signature: sm2 recover public key failed, msgHash : " + _hash.hex()));
    }
    KeyPairInterface::UniquePtr generateKeyPair() const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
    // SM2Crypto.cpp:94-122: input = hash || pub || r || s, of which the reference copies only
    // min(size, sizeof(bytesConstRef)) = 16 bytes into its struct (FixedBytes members, zero-initialised
    // by their constructors, FixedBytes.h:94); verify (the virtual) against pub, then calculateAddress =
    // right160(H(pub)); any exception -> {false, {}}.  GpuSM2Crypto overrides this with the same copy
    // (engine errors throw there).
    std::pair<bool, bytes> recoverAddress(Hash::Ptr _hashImpl, bytesConstRef _input) const override
    {
        byte in[160] = {0};
        std::memcpy(in, _input.data(), std::min(_input.size(), sizeof(_input)));
        HashType h;
        std::memcpy(h.data(), in, 32);
        bytes sig(in + 96, in + 160);
        sig.insert(sig.end(), in + 32, in + 96);
        try
        {
            auto pub = std::make_shared<KeyImpl>(64, std::make_shared<const bytes>(in + 32, in + 96));
            if (verify(pub, h, bytesConstRef(sig)))
            {
                auto d = _hashImpl->hash(bytesConstRef(pub->data()));
                return {true, bytes(d.data() + 12, d.data() + 32)};
            }
        }
        catch (...)
        {
        }
        return {false, {}};
    }
    KeyPairInterface::UniquePtr createKeyPair(SecretPtr) const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }

protected:
    std::function<int8_t(const CInputBuffer* public_key, const CInputBuffer* message_hash,
        const CInputBuffer* signature)>
        m_verifier;
};
}  // namespace crypto
}  // namespace bcos
