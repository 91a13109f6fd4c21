// mirror of bcos-crypto/signature/key/KeyImpl.h (test infrastructure, ../../../README.md)
#pragma once
#include <bcos-crypto/signature/Exceptions.h>
namespace bcos
{
namespace crypto
{
class KeyImpl : public KeyInterface
{
public:
    explicit KeyImpl(size_t _keySize) : m_keyData(std::make_shared<bytes>(_keySize)) {}
    explicit KeyImpl(size_t _keySize, std::shared_ptr<const bytes> _data) : m_keyData(std::make_shared<bytes>())
    {
        if (_data->size() < _keySize)
        {
            BOOST_THROW_EXCEPTION(InvalidKey() << errinfo_comment("invalidKey"));
        }
        *m_keyData = *_data;
    }
    const bytes& data() const override { return *m_keyData; }
    size_t size() const override { return m_keyData->size(); }
    char* mutableData() override { return (char*)m_keyData->data(); }
    const char* constData() const override { return (const char*)m_keyData->data(); }

private:
    std::shared_ptr<bytes> m_keyData;
};
}  // namespace crypto
}  // namespace bcos
