/* Reference header path -> the parsec_amd C API: scheduling (reference parsec/scheduling.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. A C++ build that sees the runtime's sources
 * (-I csrc, as parsec-ptgpp builds do) also gets the stream's fields the
 * reference's programs read: th_id, virtual_process->vp_id. */
#ifndef PARSEC_AMD_COMPAT_SCHEDULING_H
#define PARSEC_AMD_COMPAT_SCHEDULING_H
#include "../parsec.h"
#if defined(__cplusplus) && defined(__has_include)
#if __has_include("core/runtime.hpp")
#include "core/runtime.hpp"
#define parsec_execution_stream_s parsec::ExecutionStream
#endif
#endif
#endif
