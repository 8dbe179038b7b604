/* Minimal MPI for programs written against PaRSEC + MPI (the reference's
 * multi-process tests: dtd_test_pingpong / task_placement / interleave_actions
 * / explicit_task_creation, redistribute_check*.jdf, write_check.jdf,
 * multichain.jdf), implemented over this runtime's communication engine
 * (csrc/capi/mpi_shim.cpp). Build such a program with -I<repo>/include/mpi
 * -DPARSEC_HAVE_MPI and start it with `python -m parsec_amd.launch -n N`.
 *
 * What exists: init / finalize, rank / size, communicator dup / split / free,
 * barrier, bcast, reduce, allreduce, allgather on the basic C types (SUM, PROD,
 * MAX, MIN, MAXLOC, MINLOC, logical and bitwise AND / OR), MPI_IN_PLACE,
 * Wtime, Abort. Collectives are blocking and gather at the communicator's
 * first member. Point-to-point and one-sided MPI are not provided: the
 * runtime's own traffic goes through its engine. */
#ifndef PARSEC_AMD_MPI_H
#define PARSEC_AMD_MPI_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int MPI_Comm;
typedef int MPI_Datatype;
typedef int MPI_Op;
typedef long MPI_Aint;
typedef struct {
  int MPI_SOURCE, MPI_TAG, MPI_ERROR;
} MPI_Status;

#define MPI_SUCCESS 0
#define MPI_ERR_OTHER 15
#define MPI_UNDEFINED (-32766)
#define MPI_MAX_PROCESSOR_NAME 256

#define MPI_COMM_NULL ((MPI_Comm)-1)
#define MPI_COMM_WORLD ((MPI_Comm)0)
#define MPI_COMM_SELF ((MPI_Comm)1)

#define MPI_THREAD_SINGLE 0
#define MPI_THREAD_FUNNELED 1
#define MPI_THREAD_SERIALIZED 2
#define MPI_THREAD_MULTIPLE 3

#define MPI_IN_PLACE ((void*)1)

#define MPI_DATATYPE_NULL ((MPI_Datatype)0)
#define MPI_CHAR ((MPI_Datatype)1)
#define MPI_SIGNED_CHAR ((MPI_Datatype)1)
#define MPI_BYTE ((MPI_Datatype)2)
#define MPI_UNSIGNED_CHAR ((MPI_Datatype)2)
#define MPI_INT ((MPI_Datatype)3)
#define MPI_INT32_T ((MPI_Datatype)3)
#define MPI_UNSIGNED ((MPI_Datatype)4)
#define MPI_UINT32_T ((MPI_Datatype)4)
#define MPI_LONG ((MPI_Datatype)5)
#define MPI_UNSIGNED_LONG ((MPI_Datatype)6)
#define MPI_LONG_LONG_INT ((MPI_Datatype)7)
#define MPI_LONG_LONG ((MPI_Datatype)7)
#define MPI_INT64_T ((MPI_Datatype)7)
#define MPI_UNSIGNED_LONG_LONG ((MPI_Datatype)8)
#define MPI_UINT64_T ((MPI_Datatype)8)
#define MPI_FLOAT ((MPI_Datatype)9)
#define MPI_DOUBLE ((MPI_Datatype)10)
#define MPI_2INT ((MPI_Datatype)11)
#define MPI_DOUBLE_INT ((MPI_Datatype)12)
#define MPI_LONG_INT ((MPI_Datatype)13)
#define MPI_SHORT ((MPI_Datatype)14)
#define MPI_UNSIGNED_SHORT ((MPI_Datatype)15)

#define MPI_OP_NULL ((MPI_Op)0)
#define MPI_SUM ((MPI_Op)1)
#define MPI_PROD ((MPI_Op)2)
#define MPI_MAX ((MPI_Op)3)
#define MPI_MIN ((MPI_Op)4)
#define MPI_MAXLOC ((MPI_Op)5)
#define MPI_MINLOC ((MPI_Op)6)
#define MPI_LAND ((MPI_Op)7)
#define MPI_LOR ((MPI_Op)8)
#define MPI_BAND ((MPI_Op)9)
#define MPI_BOR ((MPI_Op)10)

int MPI_Init(int* argc, char*** argv);
int MPI_Init_thread(int* argc, char*** argv, int required, int* provided);
int MPI_Initialized(int* flag);
int MPI_Finalized(int* flag);
int MPI_Finalize(void);
int MPI_Abort(MPI_Comm comm, int errorcode);
int MPI_Query_thread(int* provided);
int MPI_Comm_size(MPI_Comm comm, int* size);
int MPI_Comm_rank(MPI_Comm comm, int* rank);
int MPI_Comm_dup(MPI_Comm comm, MPI_Comm* newcomm);
int MPI_Comm_split(MPI_Comm comm, int color, int key, MPI_Comm* newcomm);
int MPI_Comm_free(MPI_Comm* comm);
int MPI_Barrier(MPI_Comm comm);
int MPI_Bcast(void* buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm);
int MPI_Reduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm);
int MPI_Allreduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int MPI_Allgather(const void* sendbuf, int sendcount, MPI_Datatype sendtype, void* recvbuf, int recvcount, MPI_Datatype recvtype, MPI_Comm comm);
int MPI_Type_size(MPI_Datatype datatype, int* size);
int MPI_Get_processor_name(char* name, int* resultlen);
double MPI_Wtime(void);

#ifdef __cplusplus
}
#endif

#endif /* PARSEC_AMD_MPI_H */
