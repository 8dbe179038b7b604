/* Reference header path -> the parsec_amd C API: data collection vtable (reference parsec/data_distribution.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_DISTRIBUTION_H
#define PARSEC_AMD_COMPAT_DATA_DISTRIBUTION_H
#include "../parsec.h"
#endif
