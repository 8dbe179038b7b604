/* Reference header path -> the parsec_amd C API: 2D-cyclic vectors (reference data_dist/matrix/vector_two_dim_cyclic.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_VECTOR_TWO_DIM_CYCLIC_H
#define PARSEC_AMD_COMPAT_DATA_DIST_MATRIX_VECTOR_TWO_DIM_CYCLIC_H
#include "../../../parsec.h"
#endif
