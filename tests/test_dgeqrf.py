"""Tiled Householder QR (DGEQRF PTG taskpools): R^T R == A^T A on square, tall,
wide and ragged matrices, CPU bodies and (gpu) HIP bodies; distributed over
2 ranks on CPU. Both taskpools run: the ptgpp-compiled dgeqrf.jdf (the
benchmark's) and the hand-built C++ IR (dgeqrf.cpp, same DAG). Reference
workload: BASELINE.json config 4 (DPLASMA dgeqrf)."""
import numpy as np
import pytest


def _run_qr(pa, M, N, nb, cores=4, gpu=False, seed=0, domain=None, taskpool="jdf"):
    ctx = pa.init(cores)
    dev = pa.first_gpu_device_index() if gpu else 0
    if gpu and dev < 0:
        pytest.skip("no GPU device")
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, M, N)
    T = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, M, N)
    S = np.random.default_rng(seed).standard_normal((M, N))
    for m in range(A.mt):
        for n in range(A.nt):
            blk = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
            A.tile(m, n)[:blk.shape[0], :blk.shape[1]] = blk
    if domain is None:
        tp = pa.dgeqrf_jdf_new(A, T) if taskpool == "jdf" else pa.dgeqrf_new(A, T, 32)
    else:  # hierarchical tree: TS domains of `domain` rows, TT binary trees
        TT = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, M, N)
        tp = pa.dgeqrf_hqr_new(A, T, TT, domain)
    if not gpu:
        tp.devices_mask = 1  # CPU only
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    R = np.zeros((M, N))
    for m in range(A.mt):
        for n in range(A.nt):
            blk = R[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
            blk[:, :] = A.tile(m, n)[:blk.shape[0], :blk.shape[1]]
    ctx.fini()
    R = np.triu(R)[:min(M, N)]
    G = S.T @ S
    return np.linalg.norm(R.T @ R - G) / np.linalg.norm(G)


@pytest.mark.parametrize("taskpool", ["jdf", "ir"])
@pytest.mark.parametrize("M,N,nb", [(64, 64, 16), (80, 48, 16), (48, 80, 16), (70, 50, 16), (50, 70, 16), (96, 96, 32)])
def test_dgeqrf_cpu(pa, M, N, nb, taskpool):
    assert _run_qr(pa, M, N, nb, taskpool=taskpool) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("taskpool", ["jdf", "ir"])
@pytest.mark.parametrize("M,N,nb", [(1024, 1024, 256), (1280, 768, 256), (1000, 1000, 256), (2048, 2048, 512)])
def test_dgeqrf_gpu(pa, M, N, nb, taskpool):
    assert _run_qr(pa, M, N, nb, gpu=True, taskpool=taskpool) < 1e-12


@pytest.mark.parametrize("M,N,nb,domain", [(64, 64, 16, 1), (64, 64, 16, 2), (160, 96, 16, 3), (70, 50, 16, 2), (50, 70, 16, 2), (256, 128, 16, 4)])
def test_dgeqrf_hqr_cpu(pa, M, N, nb, domain):
    """Hierarchical QR (TS domains + TT binary trees; DPLASMA hqr): domain 1 is a
    pure binary TT tree, larger domains mix TS chains and TT merges."""
    assert _run_qr(pa, M, N, nb, domain=domain) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,nb,domain", [(2048, 2048, 256, 2), (2560, 1536, 256, 3), (2000, 2000, 256, 1)])
def test_dgeqrf_hqr_gpu(pa, M, N, nb, domain):
    """TTQRT/TTMQR on the MFMA QR kernels (zero-padded triangular staging)."""
    assert _run_qr(pa, M, N, nb, gpu=True, domain=domain) < 1e-12
