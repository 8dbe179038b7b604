/* Reference header path -> the parsec_amd C API: hash distributions (reference data_dist/hash_datadist.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_DIST_HASH_DATADIST_H
#define PARSEC_AMD_COMPAT_DATA_DIST_HASH_DATADIST_H
#include "../../parsec.h"
#endif
