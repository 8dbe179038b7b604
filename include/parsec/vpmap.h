/* Virtual-process map queries of the running context (reference parsec/vpmap.h):
 * the number of virtual processes and of threads in one of them. */
#ifndef PARSEC_VPMAP_H
#define PARSEC_VPMAP_H
#include "../parsec.h"
#ifdef __cplusplus
extern "C" {
#endif
int vpmap_get_nb_vp(void);
int vpmap_get_nb_threads_in_vp(int vp);
#ifdef __cplusplus
}
#endif
#endif
