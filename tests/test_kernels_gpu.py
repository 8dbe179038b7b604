"""Numerics of the hand-written CDNA4 fp64 tile kernels vs fp64 torch references."""
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
