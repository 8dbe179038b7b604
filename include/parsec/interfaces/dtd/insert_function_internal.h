/* Reference header path -> the parsec_amd C API: DTD internals (reference
 * interfaces/dtd/insert_function_internal.h). The reference's DTD test
 * programs include it for the public DTD calls and the diagnostics of
 * utils/debug.h; a C++ build that sees the runtime's sources (-I csrc) also
 * gets the task and stream fields they read (this_task->taskpool, es->th_id)
 * and the DTD tile's (tile->data_copy). */
#ifndef PARSEC_AMD_COMPAT_INTERFACES_DTD_INSERT_FUNCTION_INTERNAL_H
#define PARSEC_AMD_COMPAT_INTERFACES_DTD_INSERT_FUNCTION_INTERNAL_H
#include "../../../parsec.h"
#include "../../utils/debug.h"
#include "../../execution_stream.h"
#if defined(__cplusplus) && defined(__has_include)
#if __has_include("dtd/dtd.hpp")
#pragma push_macro("PASSED_BY_REF")
#undef PASSED_BY_REF /* an enumerator of the runtime's DTD header */
#include "dtd/dtd.hpp"
#pragma pop_macro("PASSED_BY_REF")
#endif
#endif
#endif
