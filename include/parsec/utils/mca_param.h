/* MCA parameters from C (reference parsec/utils/mca_param.h): registration of
 * an integer / string parameter with a default, looked up like every runtime
 * parameter (override > PARSEC_MCA_<name> > mca-params.conf > default). */
#ifndef PARSEC_AMD_COMPAT_UTILS_MCA_PARAM_H
#define PARSEC_AMD_COMPAT_UTILS_MCA_PARAM_H
#include "../../parsec.h"
#endif
