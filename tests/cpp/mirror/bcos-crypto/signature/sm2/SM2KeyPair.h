// mirror (test infrastructure, ../../../README.md)
#pragma once
namespace bcos
{
namespace crypto
{
const int SM2_PUBLIC_KEY_LEN = 64;
}
}  // namespace bcos
