/* Reference header path -> the parsec_amd C API: DTD interface (reference interfaces/dtd/insert_function.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_INTERFACES_DTD_INSERT_FUNCTION_H
#define PARSEC_AMD_COMPAT_INTERFACES_DTD_INSERT_FUNCTION_H
#include "../../../parsec.h"
#endif
