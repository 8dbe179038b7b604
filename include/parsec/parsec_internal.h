/* Reference header path -> the parsec_amd C API (reference parsec/parsec_internal.h).
 * Programs that include the reference's internal header for the task / taskpool
 * records get this runtime's: in a C++ build that sees the runtime's sources
 * (-I csrc, as parsec-ptgpp builds do) the complete execution-stream, data and
 * taskpool records; otherwise the public API of parsec.h. */
#ifndef PARSEC_AMD_COMPAT_PARSEC_INTERNAL_H
#define PARSEC_AMD_COMPAT_PARSEC_INTERNAL_H
#include "../parsec.h"
#include "execution_stream.h"
#include "data_internal.h"
#include "utils/debug.h"
#endif
