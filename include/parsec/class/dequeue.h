/* Double-ended queue (reference parsec/class/dequeue.h): a locked list usable
 * from both ends. */
#ifndef PARSEC_AMD_CLASS_DEQUEUE_H
#define PARSEC_AMD_CLASS_DEQUEUE_H
#include "list.h"
#define parsec_dequeue_push_front(d, it) parsec_list_push_front((d), (it))
#define parsec_dequeue_push_back(d, it) parsec_list_push_back((d), (it))
#define parsec_dequeue_pop_front(d) parsec_list_pop_front(d)
#define parsec_dequeue_pop_back(d) parsec_list_pop_back(d)
#define parsec_dequeue_try_pop_front(d) parsec_list_try_pop_front(d)
#define parsec_dequeue_is_empty(d) parsec_list_is_empty(d)
#define parsec_dequeue_nolock_push_front(d, it) parsec_list_nolock_push_front((d), (it))
#define parsec_dequeue_nolock_push_back(d, it) parsec_list_nolock_push_back((d), (it))
#define parsec_dequeue_nolock_pop_front(d) parsec_list_nolock_pop_front(d)
#define parsec_dequeue_nolock_pop_back(d) parsec_list_nolock_pop_back(d)
#define parsec_dequeue_nolock_is_empty(d) parsec_list_nolock_is_empty(d)
#endif
