/* Reference header path -> the parsec_amd C API: tiled matrices (reference parsec/data_dist/matrix/matrix.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_MATRIX_H
#define PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_MATRIX_H
#include "../../../parsec.h"
#endif
