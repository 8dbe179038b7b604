/* Reference header path -> the parsec_amd C API: execution streams (reference parsec/execution_stream.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_EXECUTION_STREAM_H
#define PARSEC_AMD_COMPAT_EXECUTION_STREAM_H
#include "../parsec.h"
#endif
