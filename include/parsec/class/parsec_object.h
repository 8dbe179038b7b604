/* Reference header path -> the parsec_amd C API: the object system (reference
 * parsec/class/parsec_object.h). Classes, PARSEC_OBJ_NEW / CONSTRUCT /
 * DESTRUCT / RETAIN / RELEASE are declared in parsec.h (implementation
 * csrc/capi/object.cpp); the containers live in list_item.h, list.h, lifo.h,
 * fifo.h and dequeue.h next to this file. */
#ifndef PARSEC_AMD_COMPAT_CLASS_PARSEC_OBJECT_H
#define PARSEC_AMD_COMPAT_CLASS_PARSEC_OBJECT_H
#include "../../parsec.h"
#endif
