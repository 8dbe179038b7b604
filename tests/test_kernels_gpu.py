"""Numerics of the hand-written CDNA4 fp64 tile kernels vs fp64 torch references."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("m,n,k", [(64, 64, 64), (512, 512, 512), (200, 136, 77), (1024, 1024, 1024)])
@pytest.mark.parametrize("transB", [0, 1])
def test_dgemm(pa, dev, m, n, k, transB):
    g = torch.Generator(device=dev).manual_seed(m * 7 + n + k)
    A = torch.randn((k, m), dtype=torch.float64, device=dev, generator=g).t()  # column-major m x k
    Bm = torch.randn((k, n) if transB else (n, k), dtype=torch.float64, device=dev, generator=g).t()
    C = torch.randn((n, m), dtype=torch.float64, device=dev, generator=g).t()
    Bop = Bm.t() if transB else Bm  # op(B) is k x n
    ref = -1.0 * (A @ Bop) + 0.5 * C
    rc = pa.kernel_dgemm(A.data_ptr(), Bm.data_ptr(), C.data_ptr(), m, n, k, m, Bm.stride(1), m, -1.0, 0.5, transB, 0, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    err = (C - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 1e-12, err


def test_dsyrk_lower_only(pa, dev):
    n, k = 320, 96
    A = torch.randn((k, n), dtype=torch.float64, device=dev).t()
    C = torch.randn((n, n), dtype=torch.float64, device=dev).t().contiguous().t()
    C0 = C.clone()
    pa.kernel_dgemm(A.data_ptr(), A.data_ptr(), C.data_ptr(), n, n, k, n, n, n, -1.0, 1.0, 1, 1, _stream())
    torch.cuda.synchronize()
    ref = C0 - A @ A.t()
    low = torch.tril(torch.ones(n, n, dtype=torch.bool, device=dev))
    assert (C[low] - ref[low]).abs().max().item() < 1e-11
    assert torch.equal(C[~low], C0[~low])  # upper triangle untouched


@pytest.mark.parametrize("m,n", [(512, 512), (100, 64), (1024, 256)])
def test_dtrsm(pa, dev, m, n):
    R = torch.randn((n, n), dtype=torch.float64, device=dev)
    L = torch.linalg.cholesky(R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev))
    Lc = L.t().contiguous().t()
    B = torch.randn((n, m), dtype=torch.float64, device=dev).t()
    ref = torch.linalg.solve_triangular(L, B.t(), upper=False).t()  # B L^-T
    pa.kernel_dtrsm(Lc.data_ptr(), B.data_ptr(), m, n, n, m, _stream())
    torch.cuda.synchronize()
    assert (B - ref).abs().max().item() < 1e-10


@pytest.mark.parametrize("n", [64, 512, 1000, 1024])
def test_dpotrf_tile(pa, dev, n):
    R = torch.randn((n, n), dtype=torch.float64, device=dev)
    S = R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev)
    A = S.t().contiguous().t().clone()
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    pa.kernel_dpotrf(A.data_ptr(), n, n, info.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert info.item() == 0
    L = torch.tril(A)
    err = (L @ L.t() - S).norm() / S.norm()
    assert err.item() < 1e-13


@pytest.mark.parametrize("steps", [1, 0])
@pytest.mark.parametrize("n", [128, 512, 1024])
def test_dpotrf_tile_paths_and_info(pa, dev, n, steps):
    """Both tile POTRF implementations (n/64 + 1 fused step launches, and 3
    launches per 64 columns) factor and invert the same SPD tile, and report the
    LAPACK info (first non-positive pivot, 1-based) of a tile that is not SPD."""
    prev = pa.kernel_potrf_steps(steps)
    try:
        R = torch.randn((n, n), dtype=torch.float64, device=dev)
        S = R @ R.t() / n + torch.eye(n, dtype=torch.float64, device=dev)
        A = S.t().contiguous().t().clone()
        W = _colmajor(n)
        W.fill_(3.0)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, _stream())
        torch.cuda.synchronize()
        assert info.item() == 0
        Lref = torch.linalg.cholesky(S.cpu()).to(dev)
        L = torch.tril(A)
        assert ((L - Lref).abs().max() / Lref.abs().max()).item() < 1e-12
        eye = torch.eye(n, dtype=torch.float64, device=dev)
        assert (W @ Lref - eye).abs().max().item() < 1e-10
        assert torch.triu(W, 1).abs().max().item() == 0.0
        # not SPD: a negative pivot at row 100 (1-based 101) after the leading 100 x 100
        B = S.clone()
        B[100, 100] = -1.0
        A2 = B.t().contiguous().t().clone()
        info.zero_()
        pa.kernel_dpotrf(A2.data_ptr(), n, n, info.data_ptr(), _stream())
        torch.cuda.synchronize()
        assert info.item() == 101
    finally:
        pa.kernel_potrf_steps(prev)


def _colmajor(rows, cols=None):
    cols = rows if cols is None else cols
    return torch.empty((cols, rows), dtype=torch.float64, device="cuda").t()  # rows x cols, column-major (ld = rows)


@pytest.mark.parametrize("n", [1024, 512, 320, 200])
def test_dpotrf_tile_inverse(pa, dev, n):
    """POTRF that also writes W = L^-1 by recursive doubling of the 64x64
    diagonal-block inverses (two grouped GEMMs per level); checked against the
    fp64 torch Cholesky: W L = I, W lower triangular."""
    R = torch.randn((n, n), dtype=torch.float64, device=dev)
    S = R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev)
    A = S.t().contiguous().t().clone()
    W = _colmajor(n)
    W.fill_(7.0)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    assert info.item() == 0
    L = torch.tril(A)
    assert ((L @ L.t() - S).norm() / S.norm()).item() < 1e-13
    eye = torch.eye(n, dtype=torch.float64, device=dev)
    assert (W @ L - eye).abs().max().item() < 1e-12
    assert torch.triu(W, 1).abs().max().item() == 0.0


@pytest.mark.parametrize("n,steps", [(512, 1), (1024, 1), (256, 0)])
def test_dpotrf_packed_panel_tile(pa, dev, n, steps):
    """The packed panel tile POTRF(k) sends to its TRSMs: W = L^-1 below and on
    the diagonal, L^T strictly above (written by the step kernel's LW / XW
    items; by a transpose kernel on the 3-launches-per-64-columns path)."""
    prev = pa.kernel_potrf_steps(steps)
    try:
        R = torch.randn((n, n), dtype=torch.float64, device=dev)
        S = R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev)
        A = S.t().contiguous().t().clone()
        W = _colmajor(n)
        W.fill_(7.0)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, _stream(), pack=True)
        torch.cuda.synchronize()
    finally:
        pa.kernel_potrf_steps(prev)
    assert info.item() == 0
    L = torch.tril(A)
    assert ((L @ L.t() - S).norm() / S.norm()).item() < 1e-13
    eye = torch.eye(n, dtype=torch.float64, device=dev)
    assert (torch.tril(W) @ L - eye).abs().max().item() < 1e-12
    assert torch.equal(torch.triu(W, 1), torch.triu(L.t(), 1))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("n", [512, 128])
def test_trsm_packed_panel_tile(pa, dev, mode, n):
    """Panel solve from the packed tile alone (the one tile a panel broadcast
    sends): through W (mode 0), by substitution with the L held in the tile's
    upper part (mode 2), and auto with an unknown estimate -- the device gate:
    the copy kernel estimates from the tile into workspace slots -- with the
    limit 1 (every panel by substitution); vs torch in fp64."""
    m, tasks = 384, 3
    R = torch.randn((n, n), dtype=torch.float64, device=dev)
    S = R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev)
    A = S.t().contiguous().t().clone()
    P = _colmajor(n)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), P.data_ptr(), n, _stream(), pack=True)
    torch.cuda.synchronize()
    L = torch.tril(A)
    Bs = [_colmajor(m, n) for _ in range(tasks)]
    refs = []
    for B in Bs:
        B.copy_(torch.randn((m, n), dtype=torch.float64, device=dev))
        refs.append(torch.linalg.solve_triangular(L, B.t(), upper=False).t())
    prev_limit = pa.trsm_inverse_limit()
    prev = pa.trsm_inverse_mode(mode, 1.0 if mode == 1 else 0.0)
    prev_route = pa.trsm_estimate_route(0)
    pa.trsm_estimate_stats(True)
    try:
        pa.kernel_trsm_w_batch([(B.data_ptr(), P.data_ptr(), m, n, m, n, True) for B in Bs], _stream())
        torch.cuda.synchronize()
    finally:
        pa.trsm_inverse_mode(prev, prev_limit)
        pa.trsm_estimate_route(prev_route)
    _, _, gated = pa.trsm_estimate_stats(True)
    assert gated == (tasks if mode == 1 else 0)
    for B, ref in zip(Bs, refs):
        assert ((B - ref).abs().max() / ref.abs().max()).item() < 1e-12


@pytest.mark.parametrize("m,n,tasks", [(1024, 1024, 3), (512, 512, 5), (300, 200, 2)])
def test_trsm_through_inverse(pa, dev, m, n, tasks):
    """Panel solve B := B L^-T as copy + grouped GEMM with W = L^-1 (the
    DPOTRF TRSM path) vs torch.linalg.solve_triangular in fp64."""
    R = torch.randn((n, n), dtype=torch.float64, device=dev)
    L = torch.linalg.cholesky(R @ R.t() + n * torch.eye(n, dtype=torch.float64, device=dev))
    Wt = torch.linalg.inv(L)
    W = _colmajor(n)
    W.copy_(Wt)
    Bs = [_colmajor(m, n) for _ in range(tasks)]
    refs = []
    for B in Bs:
        B.copy_(torch.randn((m, n), dtype=torch.float64, device=dev))
        refs.append(torch.linalg.solve_triangular(L, B.t(), upper=False).t())  # X L^T = B
    descs = [(B.data_ptr(), W.data_ptr(), m, n, m, n) for B in Bs]
    pa.kernel_trsm_w_batch(descs, _stream())
    torch.cuda.synchronize()
    for B, ref in zip(Bs, refs):
        assert ((B - ref).abs().max() / ref.abs().max()).item() < 1e-12


# --------------------------------------------------------------- QR kernels
def _house_qr_ref(A):
    """numpy reference of the compact-WY QR: R (upper), V (unit lower), T."""
    import numpy as np

    A = A.copy()
    m, n = A.shape
    k = min(m, n)
    V = np.zeros((m, k))
    T = np.zeros((k, k))
    for j in range(k):
        x = A[j:, j]
        alpha, sigma = x[0], float(x[1:] @ x[1:])
        if sigma == 0.0:
            tau, beta, v = 0.0, alpha, np.zeros_like(x)
            v[0] = 1.0
        else:
            beta = -np.copysign(np.sqrt(alpha * alpha + sigma), alpha)
            tau = (beta - alpha) / beta
            v = x / (alpha - beta)
            v[0] = 1.0
        A[j:, j:] -= tau * np.outer(v, v @ A[j:, j:])
        V[j:, j] = v
        T[:j, j] = -tau * T[:j, :j] @ (V[:, :j].T @ V[:, j])
        T[j, j] = tau
    return np.triu(A)[:k], V, T


def _cm(x, dev):
    """column-major device copy of a (rows, cols) array: returns the (cols, rows) tensor"""
    return torch.as_tensor(np.ascontiguousarray(np.asarray(x).T), dtype=torch.float64).to(dev)


def _np(t):
    return t.cpu().numpy().T


@pytest.mark.parametrize("m,n", [(256, 256), (300, 200), (128, 256), (512, 512), (544, 480), (232, 232), (20, 40)])
def test_qr_panel_geqrt(pa, dev, m, n):
    A = np.random.default_rng(0).standard_normal((m, n))
    k = min(m, n)
    Ad = _cm(A, dev)
    Td = torch.zeros((k, k), dtype=torch.float64, device=dev)
    Vd = torch.zeros((k, m), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert pa.kernel_qr_panel(Ad.data_ptr(), m, 0, 0, Td.data_ptr(), k, Vd.data_ptr(), m, 0, n, s) == 0
    torch.cuda.synchronize()
    R_ref, V_ref, T_ref = _house_qr_ref(A)
    assert np.allclose(np.triu(_np(Ad))[:k], R_ref, atol=1e-10)
    assert np.allclose(_np(Vd), V_ref, atol=1e-10)
    assert np.allclose(_np(Td), T_ref, atol=1e-10)


@pytest.mark.parametrize("m2,n", [(256, 256), (100, 64), (512, 512), (232, 232), (512, 200)])
def test_qr_panel_tsqrt_and_tsmqr(pa, dev, m2, n):
    rng = np.random.default_rng(1)
    R = np.triu(rng.standard_normal((n, n)))
    A2 = rng.standard_normal((m2, n))
    Rd, A2d = _cm(R, dev), _cm(A2, dev)
    Td = torch.zeros((n, n), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert pa.kernel_qr_panel(Rd.data_ptr(), n, A2d.data_ptr(), m2, Td.data_ptr(), n, 0, 0, m2, n, s) == 0
    torch.cuda.synchronize()
    R_ref, V_ref, T_ref = _house_qr_ref(np.vstack([R, A2]))
    assert np.allclose(np.triu(_np(Rd)), R_ref, atol=1e-10)
    assert np.allclose(_np(A2d), V_ref[n:], atol=1e-10)
    assert np.allclose(_np(Td), T_ref, atol=1e-10)
    # TSMQR: [B1; B2] := Q^T [B1; B2]
    nc = 96
    B1, B2 = rng.standard_normal((n, nc)), rng.standard_normal((m2, nc))
    B1d, B2d = _cm(B1, dev), _cm(B2, dev)
    ws = torch.empty(2 * n * nc, dtype=torch.float64, device=dev)
    assert pa.kernel_qr_apply(A2d.data_ptr(), m2, Td.data_ptr(), n, B1d.data_ptr(), n, B2d.data_ptr(), m2, m2, n, nc, ws.data_ptr(), s) == 0
    torch.cuda.synchronize()
    X = np.vstack([B1, B2])
    ref = X - V_ref @ (T_ref.T @ (V_ref.T @ X))
    assert np.allclose(np.vstack([_np(B1d), _np(B2d)]), ref, atol=1e-10)
