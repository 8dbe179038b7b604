/* Reference header path -> the parsec_amd C API: the object system (reference
 * parsec/class/parsec_object.h). Only the macros programs use on runtime
 * objects exist (PARSEC_OBJ_RETAIN / RELEASE / CLASS_INSTANCE, see parsec.h):
 * the runtime reference-counts its objects itself. */
#ifndef PARSEC_AMD_COMPAT_CLASS_PARSEC_OBJECT_H
#define PARSEC_AMD_COMPAT_CLASS_PARSEC_OBJECT_H
#include "../../parsec.h"
#endif
