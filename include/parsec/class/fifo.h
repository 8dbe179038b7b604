/* FIFO queue (reference parsec/class/fifo.h): a locked list, pushed at the back
 * and popped at the front. */
#ifndef PARSEC_AMD_CLASS_FIFO_H
#define PARSEC_AMD_CLASS_FIFO_H
#include "list.h"
#define parsec_fifo_push(f, it) parsec_list_push_back((f), (it))
#define parsec_fifo_pop(f) parsec_list_pop_front(f)
#define parsec_fifo_try_pop(f) parsec_list_try_pop_front(f)
#define parsec_fifo_is_empty(f) parsec_list_is_empty(f)
#define parsec_fifo_nolock_push(f, it) parsec_list_nolock_push_back((f), (it))
#define parsec_fifo_nolock_pop(f) parsec_list_nolock_pop_front(f)
#define parsec_fifo_nolock_is_empty(f) parsec_list_nolock_is_empty(f)
#endif
