/* Reference header path -> the parsec_amd C API: context / taskpool API (reference parsec/runtime.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_RUNTIME_H
#define PARSEC_AMD_COMPAT_RUNTIME_H
#include "../parsec.h"
#endif
