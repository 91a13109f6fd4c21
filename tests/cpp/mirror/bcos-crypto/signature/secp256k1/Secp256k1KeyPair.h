// mirror (test infrastructure, ../../../README.md)
#pragma once
namespace bcos
{
namespace crypto
{
const int SECP256K1_PUBLIC_LEN = 64;
}
}  // namespace bcos
