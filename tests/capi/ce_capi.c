/* The communication engine API from C: port of the reference's
 * tests/dsl/dtd/dtd_test_ce.c (active messages both ways, a GET 1 <- 0 and a
 * PUT 0 -> 1 on registered memory, completion notifications through AM tags),
 * plus pack / unpack. Two ranks (parsec_amd.launch -n 2). With "gpu" as the
 * first argument the registered buffers live in GPU memory (hipMalloc) and the
 * one-sided transfers go GPU to GPU through HIP IPC; PARSEC_COMM_GPU selects
 * the device; the GPU run then repeats both with one end in host memory (a
 * device-to-host get and a host-to-device put: the engine must use the copy
 * engines there, never a copy kernel on pageable memory). A non-contiguous
 * registration (lower triangle) is refused. Differences from the reference:
 * r_tag of get / put is an AM tag (the reference's MPI engine takes a callback
 * address); values are checked. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef CE_WITH_HIP
#include <hip/hip_runtime_api.h>
#endif

#include "parsec.h"

#define AM_FROM_0_TAG 2
#define AM_FROM_1_TAG 3
#define NOTIFY_GET_TAG 4
#define NOTIFY_PUT_TAG 5
#define MEM_HANDLE_FROM_1_TAG 6
#define GET_END_ACK_TAG 7
#define PUT_END_ACK_TAG 8
#define LATE_TAG 9 /* registered on rank 0 only after rank 1's messages arrived */
#define N 4096 /* ints per buffer: 16 KB, several ring fragments at most */

static volatile int counter = 0;
static int my_rank, use_gpu = 0, bad = 0;
/* where each end of the current phase lives (1: GPU memory) and the label */
static int get_src_gpu, get_dst_gpu, put_src_gpu, put_dst_gpu;
static const char* phase = "";
/* callbacks run on the communication thread, concurrently with main(): counter
 * is reset before each barrier, never after it */

static void* buf_alloc(size_t bytes, int gpu) {
#ifdef CE_WITH_HIP
    if (gpu) {
        void* p = NULL;
        /* a buffer object of its own (small hipMallocs can be carved out of a shared
         * one that a peer cannot attach): 64 MB, far above comm_ipc_min_alloc */
        if (hipMalloc(&p, bytes < (64u << 20) ? (64u << 20) : bytes) != hipSuccess) return NULL;
        return p;
    }
#endif
    (void)gpu;
    return malloc(bytes);
}
static void buf_free(void* p, int gpu) {
#ifdef CE_WITH_HIP
    if (gpu) { hipFree(p); return; }
#endif
    (void)gpu;
    free(p);
}
static void buf_write(void* dst, const int* src, size_t n, int gpu) {
#ifdef CE_WITH_HIP
    if (gpu) { hipMemcpy(dst, src, n * sizeof(int), hipMemcpyHostToDevice); return; }
#endif
    (void)gpu;
    memcpy(dst, src, n * sizeof(int));
}
static void buf_read(int* dst, const void* src, size_t n, int gpu) {
#ifdef CE_WITH_HIP
    if (gpu) { hipMemcpy(dst, src, n * sizeof(int), hipMemcpyDeviceToHost); return; }
#endif
    (void)gpu;
    memcpy(dst, src, n * sizeof(int));
}
static int reg(void* mem, size_t bytes, int gpu, parsec_ce_mem_reg_handle_t* h, size_t* hs) {
    if (gpu) return parsec_ce_mem_register_device(mem, bytes, parsec_ce_gpu_device_index(), h, hs);
    return parsec_ce.mem_register(mem, PARSEC_MEM_TYPE_CONTIGUOUS, 1, PARSEC_DATATYPE_NULL, bytes, h, hs);
}
static int check(const void* mem, int mult, const char* what, int gpu) {
    int* h = malloc(N * sizeof(int));
    buf_read(h, mem, N, gpu);
    int ok = 1;
    for (int i = 0; i < N; i++) if (h[i] != i * mult) { ok = 0; break; }
    printf("[%d] %s%s %s\n", my_rank, phase, what, ok ? "ok" : "WRONG");
    free(h);
    if (!ok) bad++;
    return ok;
}

static int am_ints(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)ce; (void)tag; (void)src; (void)cb_data;
    const int* v = (const int*)msg;
    if (size != 3 * sizeof(int) || v[0] != 10 || v[1] != 11 || v[2] != 12) bad++;
    counter++;
    return 1;
}
static int am_floats(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)ce; (void)tag; (void)src; (void)cb_data;
    const float* v = (const float*)msg;
    if (size != 2 * sizeof(float) || v[0] != 9.5f || v[1] != 19.5f) bad++;
    counter++;
    return 1;
}

/* ---- GET: 1 pulls from 0 */
static int get_end(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg, ptrdiff_t rdispl,
                   size_t size, int remote, void* cb_data) {
    (void)ldispl; (void)rreg; (void)rdispl; (void)remote; (void)cb_data;
    void* mem;
    parsec_datatype_t dtt;
    int count, bytes;
    ce->mem_retrieve(lreg, &mem, &dtt, &count);
    parsec_type_size(dtt, &bytes);
    if (size != N * sizeof(int) || bytes != (int)size) bad++;
    check(mem, 1, "GET", get_dst_gpu);
    ce->mem_unregister(&lreg);
    buf_free(mem, get_dst_gpu);
    counter++;
    return 1;
}
static int notify_get(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)tag; (void)size; (void)cb_data;
    /* msg = rank 0's handle; register a receive buffer and pull */
    void* rbuf = buf_alloc(N * sizeof(int), get_dst_gpu);
    parsec_ce_mem_reg_handle_t mine;
    size_t hs;
    reg(rbuf, N * sizeof(int), get_dst_gpu, &mine, &hs);
    ce->get(ce, mine, 0, (parsec_ce_mem_reg_handle_t)msg, 0, 0, src, get_end, NULL, GET_END_ACK_TAG, msg, (size_t)ce->get_mem_handle_size());
    counter++;
    return 1;
}
static int get_end_ack(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)tag; (void)size; (void)src; (void)cb_data;
    /* back on rank 0 with its own handle: release the source buffer */
    void* mem;
    ce->mem_retrieve((parsec_ce_mem_reg_handle_t)msg, &mem, NULL, NULL);
    buf_free(mem, get_src_gpu);
    counter++;
    return 1;
}

/* ---- PUT: 0 pushes into 1 */
static parsec_ce_mem_reg_handle_t put_src_handle; /* rank 0 */
static int notify_put(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)tag; (void)size; (void)cb_data;
    const int hs0 = ce->get_mem_handle_size();
    void* rbuf = buf_alloc(N * sizeof(int), put_dst_gpu);
    parsec_ce_mem_reg_handle_t mine;
    size_t hs;
    reg(rbuf, N * sizeof(int), put_dst_gpu, &mine, &hs);
    char* reply = malloc(2 * (size_t)hs0);
    memcpy(reply, msg, (size_t)hs0);                  /* 0's handle */
    memcpy(reply + hs0, mine, (size_t)hs0);           /* 1's handle */
    ce->send_am(ce, MEM_HANDLE_FROM_1_TAG, src, reply, 2 * (size_t)hs0);
    free(reply);
    counter++;
    return 1;
}
static int put_end(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg, ptrdiff_t rdispl,
                   size_t size, int remote, void* cb_data) {
    (void)ldispl; (void)rreg; (void)rdispl; (void)remote; (void)cb_data;
    if (size != N * sizeof(int)) bad++;
    void* mem;
    ce->mem_retrieve(lreg, &mem, NULL, NULL);
    ce->mem_unregister(&put_src_handle);
    buf_free(mem, put_src_gpu);
    counter++;
    return 1;
}
static int handles_from_1(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)tag; (void)size; (void)cb_data;
    const int hs = ce->get_mem_handle_size();
    parsec_ce_mem_reg_handle_t theirs = (char*)msg + hs;
    ce->put(ce, put_src_handle, 0, theirs, 0, 0, src, put_end, NULL, PUT_END_ACK_TAG, theirs, (size_t)hs);
    counter++;
    return 1;
}
static int put_end_ack(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)tag; (void)size; (void)src; (void)cb_data;
    void* mem;
    parsec_ce_mem_reg_handle_t h = (parsec_ce_mem_reg_handle_t)msg;
    ce->mem_retrieve(h, &mem, NULL, NULL);
    check(mem, 2, "PUT", put_dst_gpu);
    buf_free(mem, put_dst_gpu);
    counter++;
    return 1;
}

static void wait_for(int n) {
    while (counter < n) parsec_ce.progress(&parsec_ce);
}

/* messages on a tag registered late: delivered once it is, in send order */
static int late_next = 0;
static int late_am(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t size, int src, void* cb_data) {
    (void)ce; (void)tag; (void)cb_data;
    int v;
    memcpy(&v, msg, sizeof(v));
    if (size != sizeof(int) || src != 1 || v != late_next) {
        printf("[%d] late message %d from %d, expected %d\n", my_rank, v, src, late_next);
        bad++;
    }
    late_next++;
    counter++;
    return 1;
}

int main(int argc, char** argv) {
    use_gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    parsec_comm_engine_t* ce = parsec_comm_engine_init(NULL);
    if (!ce || ce->size != 2) {
        printf("needs 2 ranks\n");
        return 1;
    }
    my_rank = ce->rank;
    ce->tag_register(AM_FROM_0_TAG, am_ints, ce, 4096);
    ce->tag_register(AM_FROM_1_TAG, am_floats, ce, 4096);
    ce->tag_register(NOTIFY_GET_TAG, notify_get, ce, 4096);
    ce->tag_register(NOTIFY_PUT_TAG, notify_put, ce, 4096);
    ce->tag_register(MEM_HANDLE_FROM_1_TAG, handles_from_1, ce, 4096);
    ce->tag_register(GET_END_ACK_TAG, get_end_ack, ce, 4096);
    ce->tag_register(PUT_END_ACK_TAG, put_end_ack, ce, 4096);
    ce->sync(ce); /* every tag registered everywhere */

    /* active messages: 0 -> 1 twice, 1 -> 0 twice */
    if (my_rank == 0) {
        int v[3] = {10, 11, 12};
        ce->send_am(ce, AM_FROM_0_TAG, 1, v, sizeof(v));
        ce->send_am(ce, AM_FROM_0_TAG, 1, v, sizeof(v));
    } else {
        float f[2] = {9.5f, 19.5f};
        ce->send_am(ce, AM_FROM_1_TAG, 0, f, sizeof(f));
        ce->send_am(ce, AM_FROM_1_TAG, 0, f, sizeof(f));
    }
    wait_for(2);
    counter = 0; /* before the barrier: the peer's next messages may arrive right after it */
    ce->sync(ce);

    /* every end in the requested memory, then (GPU runs) one end on the host */
    for (int round = 0; round < (use_gpu ? 2 : 1); round++) {
        get_src_gpu = use_gpu;
        get_dst_gpu = use_gpu && round == 0;
        put_src_gpu = use_gpu && round == 0;
        put_dst_gpu = use_gpu;
        phase = round ? "MIXED " : "";
        /* GET: 0 registers, tells 1; 1 pulls (get_end) and acknowledges (get_end_ack on 0) */
        if (my_rank == 0) {
            int* h = malloc(N * sizeof(int));
            for (int i = 0; i < N; i++) h[i] = i;
            void* sbuf = buf_alloc(N * sizeof(int), get_src_gpu);
            buf_write(sbuf, h, N, get_src_gpu);
            free(h);
            parsec_ce_mem_reg_handle_t mine;
            size_t hs;
            reg(sbuf, N * sizeof(int), get_src_gpu, &mine, &hs);
            ce->send_am(ce, NOTIFY_GET_TAG, 1, mine, hs);
            wait_for(1);
            ce->mem_unregister(&mine);
        } else {
            wait_for(2);
        }
        counter = 0;
        ce->sync(ce);

        /* PUT: 0 tells 1, 1 answers with both handles, 0 pushes (put_end), 1 checks (put_end_ack) */
        if (my_rank == 0) {
            int* h = malloc(N * sizeof(int));
            for (int i = 0; i < N; i++) h[i] = 2 * i;
            void* sbuf = buf_alloc(N * sizeof(int), put_src_gpu);
            buf_write(sbuf, h, N, put_src_gpu);
            free(h);
            size_t hs;
            reg(sbuf, N * sizeof(int), put_src_gpu, &put_src_handle, &hs);
            ce->send_am(ce, NOTIFY_PUT_TAG, 1, put_src_handle, hs);
            wait_for(2);
        } else {
            wait_for(2);
        }
        counter = 0;
        ce->sync(ce);
    }

    /* a tag rank 0 registers only after rank 1's messages on it arrived (an MPI
     * unexpected-message queue: kept in order, not dropped) */
    if (my_rank == 1)
        for (int i = 0; i < 5; i++) ce->send_am(ce, LATE_TAG, 0, &i, sizeof(i));
    ce->sync(ce); /* rank 1's messages precede its barrier message on the same ring */
    if (my_rank == 0) {
        ce->tag_register(LATE_TAG, late_am, ce, 64);
        for (long spins = 0; counter < 5 && spins < 200000000L; spins++) parsec_ce.progress(&parsec_ce);
        if (counter != 5) {
            printf("[0] %d of 5 late-tag messages delivered\n", counter);
            bad++;
        }
    }
    counter = 0;
    ce->sync(ce);

    /* pack / unpack: the lower triangle of a 4 x 4 column-major matrix */
    {
        parsec_datatype_t lower, dbl;
        parsec_type_create_contiguous(1, parsec_datatype_double_t, &dbl);
        parsec_type_create_lower(4, 4, 1, parsec_datatype_double_t, &lower);
        double a[16], b[16] = {0};
        for (int i = 0; i < 16; i++) a[i] = i + 1;
        int psize = 0, pos = 0, upos = 0;
        ce->pack_size(ce, 1, lower, &psize);
        char* packed = malloc((size_t)psize);
        if (psize != 10 * (int)sizeof(double) || ce->pack(ce, a, 1, lower, packed, psize, &pos) != 0 || pos != psize) bad++;
        if (ce->unpack(ce, packed, psize, &upos, b, 1, lower) != 0 || upos != psize) bad++;
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                if (b[r + 4 * c] != (r >= c ? a[r + 4 * c] : 0.0)) bad++;
        free(packed);
        (void)dbl;
        /* the engine moves byte ranges: a registration whose layout is not its
         * packed image must be refused, a contiguous one accepted */
        parsec_ce_mem_reg_handle_t h;
        size_t hs;
        if (ce->mem_register(a, PARSEC_MEM_TYPE_NONCONTIGUOUS, 1, lower, sizeof(a), &h, &hs) == 0) {
            printf("[%d] non-contiguous registration accepted\n", my_rank);
            bad++;
            ce->mem_unregister(&h);
        }
        parsec_datatype_t four;
        parsec_type_create_contiguous(4, parsec_datatype_double_t, &four);
        if (ce->mem_register(a, PARSEC_MEM_TYPE_NONCONTIGUOUS, 4, four, sizeof(a), &h, &hs) != 0) bad++;
        else ce->mem_unregister(&h);
    }
    printf("[%d] ce %s (can_serve %d)\n", my_rank, bad ? "FAILED" : "ok", ce->can_serve(ce));
    ce->sync(ce);
    parsec_comm_engine_fini(ce);
    return bad ? 1 : 0;
}
