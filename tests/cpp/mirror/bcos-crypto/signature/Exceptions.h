// mirror of bcos-crypto/signature/Exceptions.h (test infrastructure, ../../README.md)
#pragma once
#include <bcos-crypto/interfaces/crypto/Signature.h>
#define BOOST_THROW_EXCEPTION(x) throw(x)
namespace bcos
{
namespace crypto
{
struct SignException : bcos::Exception {};
struct InvalidSignature : bcos::Exception {};
struct InvalidKey : bcos::Exception {};
}  // namespace crypto
}  // namespace bcos
