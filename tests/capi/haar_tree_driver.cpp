// Runs the reference's haar-tree application (tests/apps/haar_tree: project.jdf
// or project_dyn.jdf, then walk.jdf, over tree_dist.c -- all unmodified) and
// prints this rank's checksum of the built tree. The reference's main.c checks
// the XOR of the ranks' checksums against SUM_VALUE only under MPI
// (main.c:297-307); here every rank prints its own and the test combines them.
//
//   haar_tree_driver [dyn] -- <parsec args>
#include <cstdio>
#include <cstring>

#include "tree_dist.h"
#include "walk_utils.h"
#if defined(HAAR_DYN)
#include "project_dyn.h"
#define parsec_project_new parsec_project_dyn_new
#define parsec_project_taskpool_t parsec_project_dyn_taskpool_t
#define PARSEC_project_DEFAULT_ADT_IDX PARSEC_project_dyn_DEFAULT_ADT_IDX
#else
#include "project.h"
#endif
#include "walk.h"

// the reference's per-node contribution (main.c cksum_node_fn)
static void cksum_node(tree_dist_t* tree, node_t* node, int n, int l, void* param) {
  union {
    double d;
    uint64_t u;
  } a;
  int64_t* cksum = (int64_t*)param;
  int64_t up = 0;
  a.d = node->s;
  up ^= a.u;
  a.d = node->d;
  up ^= a.u;
  up ^= (((int64_t)l) << 32) | (int64_t)n;
  int64_t ov, nv;
  do {
    ov = __atomic_load_n(cksum, __ATOMIC_RELAXED);
    nv = ov ^ up;
  } while (!parsec_atomic_cas_int64(cksum, ov, nv));
  (void)tree;
}

// every node the walk goes back up through: count and XOR of the (n, l) keys
// (project_dyn.jdf also writes its leaves' NEW tiles, whose contents are not
// set, into the tree: the keys are deterministic, those contents are not)
static int nodes_up;
static int64_t keys_up;
static void count_node(tree_dist_t*, node_t*, int n, int l, void*) {
  parsec_atomic_fetch_add_int32(&nodes_up, 1);
  int64_t ov, nv;
  do {
    ov = __atomic_load_n(&keys_up, __ATOMIC_RELAXED);
    nv = ov ^ ((((int64_t)l) << 32) | (int64_t)n);
  } while (!parsec_atomic_cas_int64(&keys_up, ov, nv));
}

int main(int argc, char* argv[]) {
  int pargc = 0;
  char** pargv = nullptr;
  for (int i = 1; i < argc; i++)
    if (strcmp(argv[i], "--") == 0) {
      pargc = argc - i;
      pargv = &argv[i];
      break;
    }
  parsec_context_t* parsec = parsec_init(-1, &pargc, &pargv);
  const int rank = parsec_context_rank(parsec), world = parsec_context_nb_nodes(parsec);

  tree_dist_t* treeA = tree_dist_create_empty(rank, world);
  parsec_matrix_block_cyclic_t fakeDesc;
  parsec_matrix_block_cyclic_init(&fakeDesc, PARSEC_MATRIX_FLOAT, PARSEC_MATRIX_TILE, rank, 1, 1, world, world, 0, 0, world, world, 1, world, 1, 1, 0, 0);
  parsec_arena_datatype_t adt;
  parsec_add2arena(&adt, parsec_datatype_float_t, PARSEC_MATRIX_FULL, 0, 2, 1, 2, PARSEC_ARENA_ALIGNMENT_SSE, -1);

  const int verbose = getenv("HAAR_VERBOSE") != nullptr;
  parsec_project_taskpool_t* project = parsec_project_new(treeA, world, (parsec_data_collection_t*)&fakeDesc, 1e-3, verbose, 1.0);
  project->arenas_datatypes[PARSEC_project_DEFAULT_ADT_IDX] = adt;
  int rc = parsec_context_add_taskpool(parsec, &project->super);
  PARSEC_CHECK_ERROR(rc, "parsec_context_add_taskpool");
  rc = parsec_context_start(parsec);
  PARSEC_CHECK_ERROR(rc, "parsec_context_start");
  rc = parsec_context_wait(parsec);
  PARSEC_CHECK_ERROR(rc, "parsec_context_wait");
  parsec_taskpool_free(&project->super);

  int64_t cksum = 0;
  parsec_walk_taskpool_t* walker = parsec_walk_new(treeA, world, (parsec_data_collection_t*)&fakeDesc, &cksum, cksum_node, count_node, verbose);
  walker->arenas_datatypes[PARSEC_walk_DEFAULT_ADT_IDX] = adt;
  rc = parsec_context_add_taskpool(parsec, &walker->super);
  PARSEC_CHECK_ERROR(rc, "parsec_context_add_taskpool");
  rc = parsec_context_start(parsec);
  PARSEC_CHECK_ERROR(rc, "parsec_context_start");
  rc = parsec_context_wait(parsec);
  PARSEC_CHECK_ERROR(rc, "parsec_context_wait");
  parsec_taskpool_free(&walker->super);

  printf("haar rank %d cksum %llx nodes_up %d keys %llx\n", rank, (unsigned long long)cksum, nodes_up, (unsigned long long)keys_up);
  parsec_del2arena(&adt);
  tree_dist_free(treeA);
  parsec_fini(&parsec);
  return 0;
}
