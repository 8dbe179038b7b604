/* Machine topology queries (reference parsec/parsec_hwloc.h), from the
 * runtime's own topology discovery (sysfs, no hwloc). */
#ifndef PARSEC_AMD_COMPAT_PARSEC_HWLOC_H
#define PARSEC_AMD_COMPAT_PARSEC_HWLOC_H
#include "../parsec.h"
#endif
