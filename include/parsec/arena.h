/* Reference header path -> the parsec_amd C API: arenas (reference parsec/arena.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. Like the reference's header it brings the
 * diagnostic macros (parsec_warning, ...), and a C++ build that sees the
 * runtime's sources (-I csrc, as parsec-ptgpp builds do) gets the complete
 * arena-datatype record (adt->arena, released with PARSEC_OBJ_RELEASE). */
#ifndef PARSEC_AMD_COMPAT_ARENA_H
#define PARSEC_AMD_COMPAT_ARENA_H
#include "../parsec.h"
#include "utils/debug.h"
#if defined(__cplusplus) && defined(__has_include)
#if __has_include("core/runtime.hpp")
#include "core/runtime.hpp"
#endif
#endif
#endif
