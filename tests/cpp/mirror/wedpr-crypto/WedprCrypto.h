// mirror of wedpr-crypto's C types (test infrastructure, see ../README.md)
#pragma once
#include <stdint.h>
typedef struct { const char* data; uintptr_t len; } CInputBuffer;
typedef struct { char* data; uintptr_t len; } COutputBuffer;
#define WEDPR_SUCCESS 0
#define WEDPR_ERROR -1
