"""Views over tiled matrices (reference parsec_matrix_block_cyclic_kview,
two_dim_rectangle_cyclic.c:419-560; parsec_tiled_matrix_submatrix, matrix.c:158;
subtile_desc_create, subtile.c): ownership mapping, shared storage with the
origin, and a DTD computation through a view."""
import numpy as np


def test_kview_groups_k_rows_per_process_row(pa):
    # 2 x 1 grid, 12 tile rows; k-view with kp = 3: view rows 0..2 on process
    # row 0, 3..5 on process row 1, ... (k consecutive rows per process row)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 4, 4, 48, 8, P=2, Q=1)
    V = pa.KViewMatrix(A, 3, 1)
    ranks = [V.rank_of([m, 0]) for m in range(12)]
    assert ranks == [0, 0, 0, 1, 1, 1, 0, 0, 0, 1, 1, 1]
    # the view is a permutation of the origin's tiles
    rows = sorted(V.origin_index(m, 0)[0] for m in range(12))
    assert rows == list(range(12))
    # every view tile is the origin tile it maps to (same storage)
    for m in range(12):
        om = V.origin_index(m, 0)[0]
        if A.rank_of([om, 0]) == 0:
            A.tile(om, 0)[:, :] = 100 + m
            A.mark_host_modified(om, 0)
            assert V.tile(m, 0)[0, 0] == 100 + m
            assert V.data_key([m, 0]) == A.data_key([om, 0])


def test_kview_partial_last_group(pa):
    # 10 tile rows with P = 2, kp = 3: groups of 6, the last one partial
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 2, 2, 20, 2, P=2, Q=1)
    V = pa.KViewMatrix(A, 3, 1)
    mapped = [V.origin_index(m, 0)[0] for m in range(10)]
    assert sorted(mapped) == list(range(10))


def test_submatrix_view(pa):
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 4, 4, 16, 16)
    for m in range(4):
        for n in range(4):
            A.tile(m, n)[:, :] = 10 * m + n
            A.mark_host_modified(m, n)
    S = pa.SubMatrixView(A, 4, 8, 8, 8)  # tiles (1..2, 2..3)
    assert (S.mt, S.nt) == (2, 2)
    assert S.tile(0, 0)[0, 0] == 12 and S.tile(1, 1)[0, 0] == 23
    S.tile(1, 0)[:, :] = -1
    S.mark_host_modified(1, 0)
    assert A.tile(2, 2)[3, 3] == -1  # same storage
    assert S.data_key([1, 0]) == A.data_key([2, 2])


def test_subtile_aliases_parent_tile(pa):
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 8, 8, 16, 16)
    t = A.tile(1, 0)
    t[:, :] = np.arange(64, dtype=np.float64).reshape(8, 8, order="F")
    A.mark_host_modified(1, 0)
    S = pa.SubTileMatrix(A, 1, 0, 4, 4)
    assert (S.mt, S.nt, S.plda) == (2, 2, 8)
    # sub-tile (1, 1) is rows 4..7, cols 4..7 of the parent tile
    np.testing.assert_array_equal(S.tile(1, 1), t[4:8, 4:8])
    # a DTD task through the view writes the parent's storage
    ctx = pa.init(2)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    st = tp.tile_of(S, S.data_key([0, 1]))

    def neg(task):
        v = task.arg(0)  # 4 x 4 strided view into the parent tile
        v[:, :] *= -1
        return 0

    pa.insert_task(tp, neg, [(st, pa.INOUT)])
    tp.data_flush_all(S)
    ctx.wait()
    ctx.fini()
    np.testing.assert_array_equal(A.tile(1, 0)[0:4, 4:8], -np.arange(64, dtype=np.float64).reshape(8, 8, order="F")[0:4, 4:8])
