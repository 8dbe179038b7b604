/* Diagnostic output from C (reference parsec/utils/debug.h): warnings, info
 * and verbose debug lines to stderr, prefixed with the rank; parsec_fatal
 * aborts. The verbosity of parsec_debug_verbose follows the runtime's
 * debug_verbose MCA parameter (PARSEC_MCA_debug_verbose). */
#ifndef PARSEC_AMD_COMPAT_UTILS_DEBUG_H
#define PARSEC_AMD_COMPAT_UTILS_DEBUG_H
#include <stdio.h>
#include <stdlib.h>

#include "../../parsec.h"

#define parsec_warning(...) do { fprintf(stderr, "W@%05d ", parsec_debug_rank()); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } while (0)
#define parsec_inform(...) do { fprintf(stderr, "i@%05d ", parsec_debug_rank()); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } while (0)
#define parsec_fatal(...) do { fprintf(stderr, "X@%05d ", parsec_debug_rank()); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); abort(); } while (0)
#define parsec_debug_verbose(LVL, OUT, ...) \
  do { if ((LVL) <= parsec_debug_level()) { fprintf(stderr, "D@%05d ", parsec_debug_rank()); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } } while (0)
#define PARSEC_DEBUG_VERBOSE(LVL, OUT, ...) parsec_debug_verbose(LVL, OUT, __VA_ARGS__)
extern int parsec_debug_output;
#endif
