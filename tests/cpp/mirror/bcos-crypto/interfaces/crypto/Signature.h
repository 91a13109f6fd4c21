// mirror of the SignatureCrypto interface and the types it uses (test infrastructure, ../../../README.md)
#pragma once
#include <array>
#include <cstdint>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace bcos
{
using byte = uint8_t;
using bytes = std::vector<byte>;

class bytesConstRef  // vector_ref<const byte>
{
public:
    bytesConstRef() = default;
    bytesConstRef(const byte* _p, size_t _n) : m_p(_p), m_n(_n) {}
    bytesConstRef(const bytes& _b) : m_p(_b.data()), m_n(_b.size()) {}
    const byte* data() const { return m_p; }
    size_t size() const { return m_n; }
    bytes toBytes() const { return bytes(m_p, m_p + m_n); }

private:
    const byte* m_p = nullptr;
    size_t m_n = 0;
};

template <unsigned N>
class FixedBytes
{
public:
    enum { SIZE = N };
    byte* data() { return m_data.data(); }
    const byte* data() const { return m_data.data(); }
    std::string hex() const
    {
        static const char* d = "0123456789abcdef";
        std::string s;
        for (byte b : m_data) { s += d[b >> 4]; s += d[b & 15]; }
        return s;
    }

private:
    std::array<byte, N> m_data{};
};
using h256 = FixedBytes<32>;

// boost::exception-style streaming of errinfo_comment
struct errinfo_comment
{
    explicit errinfo_comment(std::string _s) : s(std::move(_s)) {}
    std::string s;
};
struct Exception : std::exception
{
    std::string comment;
    const char* what() const noexcept override { return comment.c_str(); }
};
template <class E, class = typename std::enable_if<std::is_base_of<Exception, E>::value>::type>
E operator<<(E _e, const errinfo_comment& _c)
{
    _e.comment = _c.s;
    return _e;
}

namespace crypto
{
using HashType = h256;

class KeyInterface
{
public:
    using Ptr = std::shared_ptr<KeyInterface>;
    virtual ~KeyInterface() {}
    virtual const bytes& data() const = 0;
    virtual size_t size() const = 0;
    virtual char* mutableData() = 0;
    virtual const char* constData() const = 0;
};
using PublicPtr = KeyInterface::Ptr;
using SecretPtr = KeyInterface::Ptr;

class KeyPairInterface
{
public:
    using UniquePtr = std::unique_ptr<KeyPairInterface>;
    virtual ~KeyPairInterface() {}
};
class Hash  // interfaces/crypto/Hash.h:37-44
{
public:
    using Ptr = std::shared_ptr<Hash>;
    virtual ~Hash() {}
    virtual HashType hash(bytesConstRef _data) = 0;
};

class SignatureCrypto
{
public:
    using Ptr = std::shared_ptr<SignatureCrypto>;
    virtual ~SignatureCrypto() = default;
    virtual std::shared_ptr<bytes> sign(
        const KeyPairInterface& _keyPair, const HashType& _hash, bool _signatureWithPub = false) const = 0;
    virtual bool verify(PublicPtr _pubKey, const HashType& _hash, bytesConstRef _signatureData) const = 0;
    virtual bool verify(std::shared_ptr<const bytes> _pubKeyBytes, const HashType& _hash,
        bytesConstRef _signatureData) const = 0;
    virtual PublicPtr recover(const HashType& _hash, bytesConstRef _signatureData) const = 0;
    virtual KeyPairInterface::UniquePtr generateKeyPair() const = 0;
    virtual std::pair<bool, bytes> recoverAddress(Hash::Ptr _hashImpl, bytesConstRef _in) const = 0;
    virtual KeyPairInterface::UniquePtr createKeyPair(SecretPtr _secretKey) const = 0;
};
}  // namespace crypto
}  // namespace bcos
