/* Wall-clock timing of the reference's tests and tools (reference
 * parsec/os-spec-timing.h): a monotonic nanosecond clock. */
#ifndef PARSEC_AMD_COMPAT_OS_SPEC_TIMING_H
#define PARSEC_AMD_COMPAT_OS_SPEC_TIMING_H
#include <stdint.h>
#include <time.h>
typedef uint64_t parsec_time_t;
static inline parsec_time_t take_time(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (parsec_time_t)ts.tv_sec * 1000000000ull + (parsec_time_t)ts.tv_nsec;
}
#define diff_time(t1, t2) ((t2) - (t1))
#define time_less(t1, t2) ((t1) < (t2))
#define TIMER_UNIT "nanosecond"
#endif
