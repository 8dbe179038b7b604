/* Runtime API entries of the reference's parsec/runtime.h, mca/device/device.c
 * and class/info.h from C: at_fini callbacks, taskpool ids (reserve / register /
 * lookup / unregister / sync), the device registry, data advice, and info
 * registries (constructor per object on first use, lookup, unregister). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

static int fini_calls = 0, bad = 0;
static int at_fini_cb(void* data) {
    if (data != &fini_calls) bad++;
    fini_calls++;
    return 0;
}

static int ctor_calls = 0, dtor_calls = 0;
static void* ctor(void* obj, void* cons_data) {
    (void)obj;
    ctor_calls++;
    int* v = malloc(sizeof(int));
    *v = *(int*)cons_data;
    return v;
}
static void dtor(void* elt, void* des_data) {
    (void)des_data;
    dtor_calls++;
    free(elt);
}

static int task_body(parsec_execution_stream_t* es, parsec_task_t* this_task) {
    (void)es; (void)this_task;
    return PARSEC_HOOK_RETURN_DONE;
}

int main(int argc, char** argv) {
    parsec_context_t* ctx = parsec_init(2, &argc, &argv);
    if (parsec_remote_dep_set_ctx(ctx, (intptr_t)42) != PARSEC_SUCCESS || parsec_remote_dep_get_ctx(ctx) != 42) bad++;
    parsec_context_at_fini(ctx, at_fini_cb, &fini_calls);

    /* taskpool ids */
    parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
    int id = parsec_taskpool_reserve_id(tp);
    if (id < 0 || parsec_taskpool_id(tp) != (uint32_t)id) bad++;
    if (parsec_taskpool_register(tp) != 0 || parsec_taskpool_lookup((uint32_t)id) != tp) bad++;
    parsec_taskpool_unregister(tp);
    if (parsec_taskpool_lookup((uint32_t)id) != NULL) bad++;
    parsec_taskpool_sync_ids();
    parsec_context_add_taskpool(ctx, tp);
    parsec_context_start(ctx);
    for (int i = 0; i < 8; i++) parsec_dtd_insert_task(tp, task_body, 0, PARSEC_DEV_CPU, "noop", PARSEC_DTD_ARG_END);
    parsec_dtd_taskpool_wait(tp);
    parsec_context_wait(ctx);
    parsec_taskpool_free(tp);

    /* devices */
    int nd = parsec_nb_devices_get();
    if (nd < 2 || parsec_device_get_type(0) != PARSEC_DEV_CPU || parsec_device_get_type(1) != PARSEC_DEV_RECURSIVE || parsec_device_get_type(nd) != PARSEC_DEV_NONE) bad++;

    /* data advice: preferred device = the CPU is accepted, an unknown device is not */
    double v = 1.0;
    parsec_data_t* holder = NULL;
    parsec_data_t* d = parsec_data_create(&holder, NULL, 7, &v, sizeof(v), PARSEC_DATA_FLAG_PARSEC_MANAGED);
    if (parsec_advise_data_on_device(d, 0, PARSEC_DEV_DATA_ADVICE_PREFERRED_DEVICE) != 0) bad++;
    if (parsec_advise_data_on_device(d, 60, PARSEC_DEV_DATA_ADVICE_PREFETCH) == 0) bad++;
    parsec_data_destroy(d);

    /* info registry */
    int seven = 7, cbd = 3;
    parsec_info_id_t iid = parsec_info_register(parsec_per_stream_infos, "test::handle", dtor, NULL, ctor, &seven, &cbd);
    void* got = NULL;
    if (iid < 0 || parsec_info_lookup(parsec_per_stream_infos, "test::handle", &got) != iid || got != &cbd) bad++;
    if (parsec_gpu_stream_info_get(iid) != NULL) bad++; /* not inside a GPU chore */
    if (parsec_info_unregister(parsec_per_stream_infos, iid, &got) != iid || got != &cbd) bad++;
    if (parsec_info_lookup(parsec_per_stream_infos, "test::handle", NULL) != -1) bad++;

    parsec_fini(&ctx);
    if (fini_calls != 1) bad++;
    printf("runtime capi %s (devices %d)\n", bad ? "FAILED" : "ok", nd);
    return bad ? 1 : 0;
}
