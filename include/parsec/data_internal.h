/* Reference header path -> the parsec_amd C API: data / data copies (reference parsec/data_internal.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_INTERNAL_H
#define PARSEC_AMD_COMPAT_DATA_INTERNAL_H
#include "../parsec.h"
#endif
