/* Driver of the reference's tests/apps/generalized_reduction/BT_reduction.jdf
 * (compiled unmodified by parsec-ptgpp; this file replaces the reference's
 * main.c + BT_reduction_wrapper.c + reduc_data.c, written against the public
 * API). The JDF reduces NT one-tile vectors of NB ints through one binary
 * tree per set bit of NT plus a linear chain across the trees; tile i starts
 * as i, so rank 0's LINEAR_REDUC(1) prints NT (NT - 1) / 2.
 * Data: NT x 1 tiles of NB ints, 1D block-cyclic over the ranks (the
 * reference's create_and_distribute_data).
 * usage: bt_reduction [NT] [NB] */
#include <stdio.h>
#include <stdlib.h>

#include "BT_reduction.h"

int main(int argc, char** argv) {
  parsec_context_t* parsec = parsec_init(2, &argc, &argv);
  const int rank = parsec_context_rank(parsec), world = parsec_context_nb_nodes(parsec);
  const int nt = argc > 1 ? atoi(argv[1]) : 7, nb = argc > 2 ? atoi(argv[2]) : 1;
  parsec_matrix_block_cyclic_t dc;
  parsec_matrix_block_cyclic_init(&dc, PARSEC_MATRIX_INTEGER, PARSEC_MATRIX_TILE, rank, nb, 1, nb * nt, 1, 0, 0, nb * nt, 1, world, 1, 1, 1, 0, 0);
  dc.mat = parsec_data_allocate((size_t)dc.super.nb_local_tiles * nb * sizeof(int));
  parsec_data_collection_set_key(&dc.super.super, "A");
  parsec_BT_reduction_taskpool_t* tp = parsec_BT_reduction_new(&dc.super, nb, nt);
  parsec_arena_datatype_construct(&tp->arenas_datatypes[PARSEC_BT_reduction_DEFAULT_ADT_IDX], nb * sizeof(int), PARSEC_ARENA_ALIGNMENT_SSE,
                                  parsec_datatype_int32_t);
  int rc = parsec_context_add_taskpool(parsec, (parsec_taskpool_t*)tp);
  PARSEC_CHECK_ERROR(rc, "parsec_context_add_taskpool");
  parsec_context_start(parsec);
  parsec_context_wait(parsec);
  parsec_taskpool_free((parsec_taskpool_t*)tp);
  parsec_data_free(dc.mat);
  parsec_tiled_matrix_destroy(&dc.super);
  if (rank == 0) printf("expected %d\n", nt * (nt - 1) / 2);
  parsec_fini(&parsec);
  return 0;
}
