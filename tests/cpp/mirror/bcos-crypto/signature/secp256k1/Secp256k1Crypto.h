// mirror of the Secp256k1Crypto class shape (test infrastructure, ../../../README.md): recover /
// verify would call wedpr (absent here), the host-side members only throw
#pragma once
#include <bcos-crypto/signature/Exceptions.h>
#include <bcos-crypto/signature/key/KeyImpl.h>
namespace bcos
{
namespace crypto
{
const int SECP256K1_SIGNATURE_LEN = 65;
class Secp256k1Crypto : public SignatureCrypto
{
public:
    Secp256k1Crypto() = default;
    ~Secp256k1Crypto() override = default;
    std::shared_ptr<bytes> sign(const KeyPairInterface&, const HashType&, bool) const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
    bool verify(PublicPtr, const HashType&, bytesConstRef) const override
    {
        throw SignException() << errinfo_comment("wedpr in the reference");
    }
    bool verify(std::shared_ptr<const bytes> _pubKeyBytes, const HashType& _hash,
        bytesConstRef _signatureData) const override
    {
        return verify(std::make_shared<KeyImpl>(64, _pubKeyBytes), _hash, _signatureData);
    }
    PublicPtr recover(const HashType&, bytesConstRef) const override
    {
        throw SignException() << errinfo_comment("wedpr in the reference");
    }
    KeyPairInterface::UniquePtr generateKeyPair() const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
    std::pair<bool, bytes> recoverAddress(Hash::Ptr, bytesConstRef) const override { return {false, {}}; }
    KeyPairInterface::UniquePtr createKeyPair(SecretPtr) const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
};
}  // namespace crypto
}  // namespace bcos
