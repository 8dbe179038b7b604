/* Reference header path -> the parsec_amd C API: band collections (reference
 * parsec/data_dist/matrix/two_dim_rectangle_cyclic_band.h). Programs written against the reference's
 * headers include this path; every declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_TWO_DIM_RECTANGLE_CYCLIC_BAND_H
#define PARSEC_AMD_COMPAT_TWO_DIM_RECTANGLE_CYCLIC_BAND_H
#include "../../../parsec.h"
#endif
