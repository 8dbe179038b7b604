/* Reference header path -> the parsec_amd C API: data / data copies (reference parsec/data_internal.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. A C++ build that sees the runtime's sources
 * (-I csrc, as parsec-ptgpp builds do) also gets the complete data / copy
 * records the reference's collections fill in by hand (copy->device_private,
 * data->device_copies[]), and PARSEC_DATA_COPY_RELEASE as in the reference. */
#ifndef PARSEC_AMD_COMPAT_DATA_INTERNAL_H
#define PARSEC_AMD_COMPAT_DATA_INTERNAL_H
#include "../parsec.h"
#if defined(__cplusplus) && defined(__has_include)
#if __has_include("core/runtime.hpp")
#include "core/runtime.hpp"
#endif
#endif
#ifndef PARSEC_DATA_COPY_RELEASE
#define PARSEC_DATA_COPY_RELEASE(c) do { parsec_data_copy_release(c); (c) = NULL; } while (0)
#endif
#endif
