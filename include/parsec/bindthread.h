/* Thread binding (reference parsec/bindthread.h): pin the calling thread to a
 * core (ht: hyper-thread index, ignored -- one hardware thread per core id). */
#ifndef PARSEC_AMD_COMPAT_BINDTHREAD_H
#define PARSEC_AMD_COMPAT_BINDTHREAD_H
#include "../parsec.h"
#endif
