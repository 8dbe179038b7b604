/* Reference header path -> the parsec_amd C API: build configuration (reference parsec/parsec_config.h): this runtime has no MPI; HIP is its device module.
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_PARSEC_CONFIG_H
#define PARSEC_AMD_COMPAT_PARSEC_CONFIG_H
#include "../parsec.h"
#define PARSEC_HAVE_HIP 1
#ifndef PARSEC_DECLSPEC
#define PARSEC_DECLSPEC /* symbols are exported by default */
#endif
#define PARSEC_DIST_COLLECTIVES 1
/* glibc provides getopt.h and getopt_long (reference CMake checks PARSEC_HAVE_GETOPT_H / _LONG) */
#define PARSEC_HAVE_GETOPT_H 1
#define PARSEC_HAVE_GETOPT_LONG 1
#endif
