/* Reference header path -> the parsec_amd C API: tabular matrices (reference data_dist/matrix/two_dim_tabular.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_TWO_DIM_TABULAR_H
#define PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_TWO_DIM_TABULAR_H
#include "../../../parsec.h"
#endif
