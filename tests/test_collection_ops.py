"""Built-in collection taskpools (apply / map / reduce / broadcast /
redistribute) and tiled DGEMM (PTG and DTD) on CPU; reference
data_dist/matrix/*.jdf, tests/collections/{reduce,redistribute}, and
tests/dsl/dtd/dtd_test_simple_gemm.c (BASELINE config 1: DTD tiled DGEMM)."""
import numpy as np
import pytest


def _mat(pa, M, N, mb, nb=None, fill=None, seed=0, P=1, Q=1):
    nb = nb or mb
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, mb, nb, M, N, P=P, Q=Q)
    S = np.random.default_rng(seed).standard_normal((M, N)) if fill is None else np.full((M, N), float(fill))
    for m in range(A.mt):
        for n in range(A.nt):
            blk = S[m * mb:(m + 1) * mb, n * nb:(n + 1) * nb]
            A.tile(m, n)[:blk.shape[0], :blk.shape[1]] = blk
    return A, S


def _dense(A, M, N, mb, nb=None):
    nb = nb or mb
    R = np.zeros((M, N))
    for m in range(A.mt):
        for n in range(A.nt):
            blk = R[m * mb:(m + 1) * mb, n * nb:(n + 1) * nb]
            blk[:, :] = A.tile(m, n)[:blk.shape[0], :blk.shape[1]]
    return R


def _run(pa, ctx, tp):
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()


def test_apply_lower(pa):
    ctx = pa.init(3)
    A, S = _mat(pa, 40, 40, 8)
    seen = []
    _run(pa, ctx, pa.apply_new(A, pa.MATRIX_LOWER, lambda m, n, t: (seen.append((m, n)), t.__imul__(2.0))))
    R = _dense(A, 40, 40, 8)
    for m in range(5):
        for n in range(5):
            blk = R[m * 8:(m + 1) * 8, n * 8:(n + 1) * 8]
            assert np.allclose(blk, S[m * 8:(m + 1) * 8, n * 8:(n + 1) * 8] * (2.0 if m >= n else 1.0))
    assert sorted(seen) == sorted((m, n) for m in range(5) for n in range(5) if m >= n)
    ctx.fini()


def test_map_operator(pa):
    ctx = pa.init(3)
    A, S = _mat(pa, 30, 20, 8)
    B, _ = _mat(pa, 30, 20, 8, fill=0)

    def f(src, dst, m, n):
        dst[:, :] = src * src + m

    _run(pa, ctx, pa.map_new(A, B, f))
    R = _dense(B, 30, 20, 8)
    ref = S * S + (np.arange(30) // 8)[:, None]
    assert np.allclose(R, ref)
    ctx.fini()


@pytest.mark.parametrize("by_col", [True, False])
@pytest.mark.parametrize("native", [True, False])
def test_reduce(pa, by_col, native):
    ctx = pa.init(3)
    M, N, b = 32, 24, 8
    A, S = _mat(pa, M, N, b)
    res, _ = _mat(pa, b if by_col else M, N if by_col else b, b, fill=0)

    def add(inp, io, first):
        if first:
            io[:, :] = inp
        else:
            io += inp

    tp = (pa.reduce_col_new if by_col else pa.reduce_row_new)(A, res, "sum" if native else add)
    _run(pa, ctx, tp)
    if by_col:
        got = _dense(res, b, N, b)
        ref = S.reshape(M // b, b, N).sum(axis=0)
    else:
        got = _dense(res, M, b, b)
        ref = S.reshape(M, N // b, b).sum(axis=1)
    assert np.allclose(got, ref)
    ctx.fini()


def test_broadcast(pa):
    ctx = pa.init(3)
    A, S = _mat(pa, 24, 24, 8)
    D, _ = _mat(pa, 32, 16, 8, fill=0)
    _run(pa, ctx, pa.broadcast_new(A, 1, 2, D))
    R = _dense(D, 32, 16, 8)
    src = S[8:16, 16:24]
    for m in range(4):
        for n in range(2):
            assert np.allclose(R[m * 8:(m + 1) * 8, n * 8:(n + 1) * 8], src)
    ctx.fini()


@pytest.mark.parametrize("smb,dmb", [(8, 8), (8, 5), (6, 11)])
def test_redistribute(pa, smb, dmb):
    ctx = pa.init(3)
    Sm, Sd = _mat(pa, 40, 36, smb, seed=1)
    Dm, Dd = _mat(pa, 44, 40, dmb, seed=2)
    pa.redistribute(ctx, Sm, Dm, 17, 13, 3, 5, 9, 2)
    got = _dense(Dm, 44, 40, dmb)
    ref = Dd.copy()
    ref[9:9 + 17, 2:2 + 13] = Sd[3:3 + 17, 5:5 + 13]
    assert np.allclose(got, ref)
    ctx.fini()


@pytest.mark.parametrize("transB", [0, 1])
def test_ptg_dgemm(pa, transB):
    ctx = pa.init(4)
    M, N, K, b = 40, 24, 32, 8
    A, SA = _mat(pa, M, K, b, seed=3)
    B, SB = _mat(pa, N, K, b, seed=4) if transB else _mat(pa, K, N, b, seed=4)
    C, SC = _mat(pa, M, N, b, seed=5)
    tp = pa.dgemm_new(1.5, A, B, 0.5, C, transB)
    tp.devices_mask = 1
    _run(pa, ctx, tp)
    ref = 1.5 * SA @ (SB.T if transB else SB) + 0.5 * SC
    assert np.allclose(_dense(C, M, N, b), ref)
    ctx.fini()


@pytest.mark.parametrize("transB", [0, 1])
@pytest.mark.parametrize("b", [50, 300])
def test_ptg_dgemm_host_kernel_edges(pa, b, transB):
    """Tiles large enough for the packed host GEMM (csrc/algos/host_gemm.cpp:
    24 x 8 AVX-512 / 8 x 4 AVX2 register tiles): b = 50 leaves 2-row / 2-column
    edge tiles, b = 300 spans two k blocks (KC 256) and three row blocks."""
    ctx = pa.init(4)
    M, N, K = 2 * b, b, 2 * b
    A, SA = _mat(pa, M, K, b, seed=13)
    B, SB = _mat(pa, N, K, b, seed=14) if transB else _mat(pa, K, N, b, seed=14)
    C, SC = _mat(pa, M, N, b, seed=15)
    tp = pa.dgemm_new(-0.75, A, B, 1.0, C, transB)
    tp.devices_mask = 1
    _run(pa, ctx, tp)
    ref = -0.75 * SA @ (SB.T if transB else SB) + SC
    assert np.allclose(_dense(C, M, N, b), ref, rtol=1e-12, atol=1e-11)
    ctx.fini()


def test_dtd_dgemm_4x4_tiles(pa):
    """BASELINE config 1: DTD tiled DGEMM, 4x4 tiles, one CPU process."""
    ctx = pa.init(4)
    b = 16
    A, SA = _mat(pa, 4 * b, 4 * b, b, seed=6)
    B, SB = _mat(pa, 4 * b, 4 * b, b, seed=7)
    C, SC = _mat(pa, 4 * b, 4 * b, b, seed=8)
    pa.dtd_dgemm(ctx, 1.0, A, B, 1.0, C, False)
    assert np.allclose(_dense(C, 4 * b, 4 * b, b), SA @ SB + SC)
    ctx.fini()


@pytest.mark.gpu
def test_ptg_dgemm_gpu(pa):
    ctx = pa.init(4)
    if pa.first_gpu_device_index() < 0:
        pytest.skip("no GPU")
    M, N, K, b = 1024, 768, 1280, 256
    A, SA = _mat(pa, M, K, b, seed=3)
    B, SB = _mat(pa, K, N, b, seed=4)
    C, SC = _mat(pa, M, N, b, seed=5)
    _run(pa, ctx, pa.dgemm_new(1.0, A, B, 1.0, C, 0))
    assert np.allclose(_dense(C, M, N, b), SA @ SB + SC)
    ctx.fini()


def test_tiled_matrix_data_write_read(pa, tmp_path):
    """parsec_tiled_matrix_data_write / _read (reference data_dist/matrix/matrix.h:133-135):
    local tiles dumped after a DAG ran on them, reloaded into a fresh collection;
    a file written with another tiling is refused."""
    import numpy as np

    ctx = pa.init(2)
    nb, N = 16, 40
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
    rng = np.random.default_rng(3)
    ref = {}
    for m in range(A.mt):
        for n in range(A.nt):
            ref[m, n] = rng.standard_normal((nb, nb))
            A.tile(m, n)[:, :] = ref[m, n]
    path = str(tmp_path / "A.bin")
    assert A.data_write(path) == 0
    B = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
    for m in range(B.mt):
        for n in range(B.nt):
            B.tile(m, n)[:, :] = 0.0
    assert B.data_read(path) == 0
    for (m, n), t in ref.items():
        assert np.array_equal(np.asarray(B.tile(m, n)), t)
    C = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 8, 8, N, N)
    assert C.data_read(path) != 0
    assert B.data_read(str(tmp_path / "missing.bin")) != 0
    ctx.fini()


@pytest.mark.parametrize("pad", [False, True])
def test_diag_band_to_rect(pa, pad):
    """Diagonal + sub-diagonal tiles to LAPACK band storage (reference
    data_dist/matrix/diag_band_to_rect.jdf), checked against numpy."""
    ctx = pa.init(2)
    nb, NT = 6, 5
    A, S = _mat(pa, nb * NT, nb * NT, nb, seed=7)
    ncols = (NT + (1 if pad else 0)) * (nb + 2)
    B = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb + 1, nb + 2, nb + 1, ncols)
    for n in range(B.nt):
        B.tile(0, n)[:, :] = 7.0
    _run(pa, ctx, pa.diag_band_to_rect_new(A, B, NT, NT, nb, nb))
    for k in range(B.nt):
        got = B.tile(0, k)
        want = np.zeros((nb + 1, nb + 2))
        if k < NT:
            for j in range(nb):
                col = k * nb + j
                for i in range(nb + 1):
                    r = col + i
                    # entries below the band's last tile are zero
                    want[i, j] = S[r, col] if r < nb * NT and (r // nb) <= k + 1 and (k < NT - 1 or r // nb == k) else 0.0
        assert np.array_equal(got, want), (k, got, want)
    ctx.fini()


def test_redistribute_ptg_and_dtd_agree(pa):
    """The PTG (default) and DTD forms produce the same target."""
    outs = []
    for method in ("ptg", "dtd"):
        ctx = pa.init(3)
        Sm, Sd = _mat(pa, 40, 36, 7, seed=1)
        Dm, Dd = _mat(pa, 44, 40, 5, seed=2)
        pa.redistribute(ctx, Sm, Dm, 20, 17, 1, 4, 6, 9, method=method)
        outs.append(_dense(Dm, 44, 40, 5))
        ctx.fini()
    assert np.array_equal(outs[0], outs[1])
