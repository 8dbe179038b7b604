/* Thread barrier of the public class API (reference parsec/class/barrier.h):
 * the POSIX barrier. */
#ifndef PARSEC_AMD_COMPAT_CLASS_BARRIER_H
#define PARSEC_AMD_COMPAT_CLASS_BARRIER_H
#include <pthread.h>
typedef pthread_barrier_t parsec_barrier_t;
#define parsec_barrier_init(b, attr, count) pthread_barrier_init((b), (attr), (unsigned)(count))
#define parsec_barrier_wait(b) pthread_barrier_wait(b)
#define parsec_barrier_destroy(b) pthread_barrier_destroy(b)
#endif
