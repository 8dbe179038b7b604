/* Reference header path -> the parsec_amd C API: tracing (reference parsec/profiling.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_PROFILING_H
#define PARSEC_AMD_COMPAT_PROFILING_H
#include "../parsec.h"
#endif
