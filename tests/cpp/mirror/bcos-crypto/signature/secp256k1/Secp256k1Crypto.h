// mirror of the Secp256k1Crypto class shape (test infrastructure, ../../../README.md): recover /
// verify would call wedpr (absent here), the host-side members only throw
#pragma once
#include <bcos-crypto/signature/Exceptions.h>
#include <bcos-crypto/signature/key/KeyImpl.h>
#include <bcos-crypto/signature/secp256k1/Secp256k1KeyPair.h>
namespace bcos
{
namespace crypto
{
const int SECP256K1_SIGNATURE_LEN = 65;
// the free functions over wedpr (Secp256k1Crypto.cpp:51-63, 79-124): absent here, so they throw
inline bool secp256k1Verify(PublicPtr, const HashType&, bytesConstRef)
{
    throw SignException() << errinfo_comment("wedpr_secp256k1_verify in the reference");
}
inline std::pair<bool, bytes> secp256k1Recover(Hash::Ptr, bytesConstRef)
{
    throw SignException() << errinfo_comment("wedpr_secp256k1_recover_public_key in the reference");
}
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
    // Secp256k1Crypto.cpp:126-131: the FREE function, not the virtual overload above
    bool verify(std::shared_ptr<const bytes> _pubKeyBytes, const HashType& _hash,
        bytesConstRef _signatureData) const override
    {
        return secp256k1Verify(
            std::make_shared<KeyImpl>(SECP256K1_PUBLIC_LEN, _pubKeyBytes), _hash, _signatureData);
    }
    PublicPtr recover(const HashType&, bytesConstRef) const override
    {
        throw SignException() << errinfo_comment("wedpr in the reference");
    }
    KeyPairInterface::UniquePtr generateKeyPair() const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
    // Secp256k1Crypto.h:66-69 -> the free secp256k1Recover(hashImpl, input)
    std::pair<bool, bytes> recoverAddress(Hash::Ptr _hashImpl, bytesConstRef _in) const override
    {
        return secp256k1Recover(_hashImpl, _in);
    }
    KeyPairInterface::UniquePtr createKeyPair(SecretPtr) const override
    {
        throw SignException() << errinfo_comment("host-side (wedpr) in the reference");
    }
};
}  // namespace crypto
}  // namespace bcos
