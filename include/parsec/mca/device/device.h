/* Device modules as user collections see them (reference parsec/mca/device/device.h):
 * a collection's register_memory / unregister_memory hooks receive one and call its
 * memory_register / memory_unregister to pin their storage for transfers. This
 * runtime stages host tiles through its own pinned buffers and never requires
 * the registration: the hooks are kept so that collections which set them
 * compile and behave as a no-op registration. */
#ifndef PARSEC_MCA_DEVICE_DEVICE_H
#define PARSEC_MCA_DEVICE_DEVICE_H
#include "../../../parsec.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct parsec_device_module_s parsec_device_module_t;
struct parsec_device_module_s {
  const char* name;
  uint32_t type;       /* PARSEC_DEV_CPU / PARSEC_DEV_HIP / ... */
  int device_index;    /* runtime device index */
  int (*memory_register)(parsec_device_module_t* device, parsec_data_collection_t* dc, void* ptr, size_t length);
  int (*memory_unregister)(parsec_device_module_t* device, parsec_data_collection_t* dc, void* ptr);
};
#ifdef __cplusplus
}
#endif
#endif
