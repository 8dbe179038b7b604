/* Tiled-matrix checkpoint through the C API with user storage assigned AFTER
 * init (the reference's usual pattern: parsec_matrix_block_cyclic_init, then
 * dc.mat = ...): data_write / data_read must pick the storage up lazily, and
 * set_storage_device must refuse a matrix that already owns user storage.
 * Reference: parsec/data_dist/matrix/matrix.c:269-290 (dc->data_of). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

#define MB 8
#define NTILES 4

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  parsec_context_t* ctx = parsec_init(1, &argc, &argv);
  parsec_matrix_block_cyclic_t A;
  const int N = MB * NTILES;
  parsec_matrix_block_cyclic_init(&A, PARSEC_MATRIX_DOUBLE, PARSEC_MATRIX_TILE, 0, MB, MB, N, N, 0, 0, N, N, 1, 1, 1, 1, 0, 0);
  double* mat = (double*)parsec_data_allocate(sizeof(double) * N * N);
  for (int i = 0; i < N * N; ++i) mat[i] = 0.5 * i + 1.0;
  A.mat = mat; /* assigned after init, never touched through data_of yet */
  if (parsec_tiled_matrix_set_storage_device(&A.super, 2) == PARSEC_SUCCESS) { printf("set_storage_device accepted a user-owned matrix\n"); return 1; }
  if (parsec_tiled_matrix_data_write(&A.super, argv[1]) != PARSEC_SUCCESS) { printf("write failed\n"); return 1; }
  memset(mat, 0, sizeof(double) * N * N);
  if (parsec_tiled_matrix_data_read(&A.super, argv[1]) != PARSEC_SUCCESS) { printf("read failed\n"); return 1; }
  int bad = 0;
  for (int i = 0; i < N * N; ++i) bad += mat[i] != 0.5 * i + 1.0;
  parsec_tiled_matrix_destroy(&A.super);
  parsec_data_free(mat);
  parsec_fini(&ctx);
  printf("bad %d\n%s\n", bad, bad ? "FAIL" : "ok");
  return bad != 0;
}
