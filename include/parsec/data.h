/* Reference header path -> the parsec_amd C API: data / data copies (reference parsec/data.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_H
#define PARSEC_AMD_COMPAT_DATA_H
#include "../parsec.h"
#endif
