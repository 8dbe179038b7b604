/* Reference header path -> the parsec_amd C API: datatypes (reference parsec/datatype.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATATYPE_H
#define PARSEC_AMD_COMPAT_DATATYPE_H
#include "../parsec.h"
#endif
