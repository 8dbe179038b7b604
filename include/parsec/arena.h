/* Reference header path -> the parsec_amd C API: arenas (reference parsec/arena.h).
 * Programs written against the reference's headers include this path; every
 * declaration lives in parsec.h. */
#ifndef PARSEC_AMD_COMPAT_ARENA_H
#define PARSEC_AMD_COMPAT_ARENA_H
#include "../parsec.h"
#endif
