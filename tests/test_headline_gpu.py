"""The exact kernels and configuration behind the headline number, checked
against fp64 torch references:

* the grouped 128x128 8-wave DGEMM in its FULL / C-preload form (selected only
  when a launch holds >= 384 128-tiles: tile_kernels.hip launch_gemm_chunk), for
  the GEMM (NT, alpha=-1, beta=1) and lower-only SYRK descriptors DPOTRF emits;
* tiled DPOTRF at nb=1024 (grouped batches of >= 384 tiles) on an
  ill-conditioned SPD matrix A = Q diag(lambda) Q^T, cond(A) = 1e10, not
  diagonally dominant, with the default panel solve through W = L^-1 and with
  the blocked TRSM (dpotrf_trsm_inverse=0).

Validation pattern: reference tests/dsl/dtd/dtd_test_simple_gemm.c:557-666
(compute, then validate against a reference computation).
"""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _cm(rows, cols, dev, gen):
    """rows x cols column-major fp64 matrix (ld = rows)"""
    return torch.randn((cols, rows), dtype=torch.float64, device=dev, generator=gen).t()


def test_dgemm_batch_128_full_preload(pa):
    """8 descriptors of 1024^3 (8 x 64 = 512 128-tiles >= 384): big FULL kernel
    with the accumulators preloaded from C (|alpha| = 1)."""
    dev = _dev()
    g = torch.Generator(device=dev).manual_seed(11)
    n, cnt = 1024, 8
    As = [_cm(n, n, dev, g) for _ in range(cnt)]
    Bs = [_cm(n, n, dev, g) for _ in range(cnt)]
    Cs = [_cm(n, n, dev, g) for _ in range(cnt)]
    refs = [C - A @ B.t() for A, B, C in zip(As, Bs, Cs)]
    descs = [(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, 0) for A, B, C in zip(As, Bs, Cs)]
    assert pa.kernel_dgemm_batch(descs, _stream()) == 0
    torch.cuda.synchronize()
    for C, ref in zip(Cs, refs):
        err = ((C - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-14, err


def test_dgemm_batch_128_mixed_syrk_gemm(pa):
    """The DPOTRF trailing-update mix in one launch: lower-only SYRK tiles (C = C -
    A A^T, upper triangle untouched) next to GEMM tiles, beta=1, alpha=-1."""
    dev = _dev()
    g = torch.Generator(device=dev).manual_seed(12)
    n = 1024
    descs, checks = [], []
    for i in range(7):
        A = _cm(n, n, dev, g)
        C = _cm(n, n, dev, g)
        C0 = C.clone()
        if i % 2 == 0:  # SYRK
            descs.append((A.data_ptr(), A.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, 1))
            checks.append(("syrk", C, C0 - A @ A.t(), C0, A))
        else:
            B = _cm(n, n, dev, g)
            descs.append((A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, 0))
            checks.append(("gemm", C, C0 - A @ B.t(), C0, (A, B)))
    assert pa.kernel_dgemm_batch(descs, _stream()) == 0
    torch.cuda.synchronize()
    low = torch.tril(torch.ones(n, n, dtype=torch.bool, device=dev))
    for kind, C, ref, C0, _ in checks:
        if kind == "syrk":
            assert ((C[low] - ref[low]).abs().max() / ref[low].abs().max()).item() < 1e-14
            assert torch.equal(C[~low], C0[~low])
        else:
            assert ((C - ref).abs().max() / ref.abs().max()).item() < 1e-14


@pytest.mark.parametrize("syrk", [False, True])
def test_dgemm_batch_split_k_tail(pa, syrk):
    """9 descriptors of 1024^3 = 576 128-tiles on 512 resident slots: the 64 tiles
    of the second round are split 4 ways along K and accumulated into C with f64
    atomics (beta = 1); every element must match the fp64 reference."""
    dev = _dev()
    g = torch.Generator(device=dev).manual_seed(21)
    n, cnt = 1024, 9
    As = [_cm(n, n, dev, g) for _ in range(cnt)]
    Bs = As if syrk else [_cm(n, n, dev, g) for _ in range(cnt)]
    Cs = [_cm(n, n, dev, g) for _ in range(cnt)]
    C0 = [C.clone() for C in Cs]
    refs = [C - A @ B.t() for A, B, C in zip(As, Bs, Cs)]
    descs = [(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, int(syrk)) for A, B, C in zip(As, Bs, Cs)]
    prev = pa.kernel_gemm_splitk(1)
    try:
        assert pa.kernel_dgemm_batch(descs, _stream()) == 0
        torch.cuda.synchronize()
    finally:
        pa.kernel_gemm_splitk(prev)
    low = torch.tril(torch.ones(n, n, dtype=torch.bool, device=dev))
    for C, ref, c0 in zip(Cs, refs, C0):
        if syrk:
            assert ((C[low] - ref[low]).abs().max() / ref[low].abs().max()).item() < 1e-14
            assert torch.equal(C[~low], c0[~low])
        else:
            assert ((C - ref).abs().max() / ref.abs().max()).item() < 1e-14


def test_dgemm_batch_big_tiles_forced_edge(pa):
    """128x128 kernel on ragged shapes (non-FULL path with bounds checks)."""
    dev = _dev()
    prev = pa.kernel_gemm_tile_policy(128)
    try:
        g = torch.Generator(device=dev).manual_seed(13)
        m, n, k = 1000, 904, 1000
        A, B, C = _cm(m, k, dev, g), _cm(n, k, dev, g), _cm(m, n, dev, g)
        ref = C - A @ B.t()
        assert pa.kernel_dgemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), m, n, k, m, n, m, -1.0, 1.0, 1, 0, _stream()) == 0
        torch.cuda.synchronize()
        assert ((C - ref).abs().max() / ref.abs().max()).item() < 1e-14
    finally:
        pa.kernel_gemm_tile_policy(prev)


def _illcond_spd(N, cond, dev, seed=5):
    g = torch.Generator(device=dev).manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn((N, N), dtype=torch.float64, device=dev, generator=g))
    lam = torch.logspace(0, -torch.log10(torch.tensor(float(cond))).item(), N, dtype=torch.float64, device=dev)
    S = (Q * lam) @ Q.t()
    return (S + S.t()) / 2


@pytest.mark.parametrize("trsm_inverse", ["1", "0"])
def test_dpotrf_illconditioned_nb1024(pa, trsm_inverse):
    """N=8192, nb=1024: every trailing update batch reaches the big GEMM kernel;
    backward error and forward error against torch.linalg.cholesky."""
    dev = _dev()
    N, nb = 8192, 1024
    NT = N // nb
    S = _illcond_spd(N, 1e10, dev)
    pa.mca_set("dpotrf_trsm_inverse", trsm_inverse)
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device=dev)
        store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        torch.cuda.synchronize()
        tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        assert pa.read_int(info) == 0
        L = torch.tril(store.permute(1, 3, 0, 2).reshape(N, N))
        backward = (torch.linalg.norm(L @ L.t() - S) / torch.linalg.norm(S)).item()
        Lref = torch.linalg.cholesky(S.cpu()).to(dev)  # host LAPACK oracle
        backward_ref = (torch.linalg.norm(Lref @ Lref.t() - S) / torch.linalg.norm(S)).item()
        forward = (torch.linalg.norm(L - Lref) / torch.linalg.norm(Lref)).item()
        print(f"trsm_inverse={trsm_inverse} backward={backward:.3e} (torch {backward_ref:.3e}) forward-vs-torch={forward:.3e}")
        # backward stable like the library factorization (within a small factor)
        assert backward < max(20 * backward_ref, 1e-15), (backward, backward_ref)
        # forward difference bounded by cond(A) * eps
        assert forward < 1e-4, forward
    finally:
        ctx.fini()
        pa.mca_unset("dpotrf_trsm_inverse")


@pytest.mark.parametrize("N,nb", [(4096, 512), (8192, 1024)])
def test_dpotrf_jdf_gpu(pa, N, nb):
    """The ptgpp-compiled dpotrf_L.jdf with its BODY [type = HIP] chores on the
    MI355X (same batched kernels as the C++ IR taskpool), host LAPACK oracle."""
    dev = _dev()
    NT = N // nb
    S = _illcond_spd(N, 1e6, dev, seed=8)
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device=dev)
        store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        torch.cuda.synchronize()
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        assert pa.read_int(info) == 0
        stats = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]
        assert stats["executed_tasks"] > 0
        L = torch.tril(store.permute(1, 3, 0, 2).reshape(N, N))
        backward = (torch.linalg.norm(L @ L.t() - S) / torch.linalg.norm(S)).item()
        Lref = torch.linalg.cholesky(S.cpu()).to(dev)
        backward_ref = (torch.linalg.norm(Lref @ Lref.t() - S) / torch.linalg.norm(S)).item()
        print(f"jdf N={N} nb={nb} backward={backward:.3e} (torch {backward_ref:.3e})")
        assert backward < max(20 * backward_ref, 1e-15)
    finally:
        ctx.fini()
