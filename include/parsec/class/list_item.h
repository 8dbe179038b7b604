/* Items of the public containers (reference parsec/class/list_item.h): an
 * object with a doubly linked pair of links. A C "subclass" embeds it first
 * (struct { parsec_list_item_t super; ... }). */
#ifndef PARSEC_AMD_CLASS_LIST_ITEM_H
#define PARSEC_AMD_CLASS_LIST_ITEM_H
#include "../../parsec.h"
#ifdef __cplusplus
extern "C" {
#endif
struct parsec_list_item_s {
  parsec_object_t super;
  volatile struct parsec_list_item_s* list_next;
  volatile struct parsec_list_item_s* list_prev;
  int32_t aba_key;
  int32_t reserved;
};
#define PARSEC_LIST_ITEM_NEXT(item) ((parsec_list_item_t*)((parsec_list_item_t*)(item))->list_next)
#define PARSEC_LIST_ITEM_PREV(item) ((parsec_list_item_t*)((parsec_list_item_t*)(item))->list_prev)
#ifdef __cplusplus
}
#endif
#endif
