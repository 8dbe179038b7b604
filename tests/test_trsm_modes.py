"""Panel solve of the JDF Cholesky (csrc/algos/jdf/dpotrf_L.jdf TRSM): through
W = L(k,k)^-1 (mode 0), auto (mode 1, the default: substitution with L(k,k)
when max|L(k,k)| * max|W| exceeds the limit), or always by substitution
(mode 2). CPU bodies; the GPU kernels are checked by
tests/test_dpotrf_gpu.py::test_trsm_inverse_modes_gpu. Numerics behind the
default limit: profiles/r4_trsm_inverse_numerics.txt."""
import numpy as np
import pytest


def _run(pa, S, N, nb, mode, limit=0.0):
    prev_limit = pa.trsm_inverse_limit()
    prev = pa.trsm_inverse_mode(mode, limit)
    try:
        ctx = pa.init(4)
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
        for m in range(A.mt):
            for n in range(A.nt):
                A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        L = np.zeros((N, N))
        for m in range(A.mt):
            for n in range(m + 1):
                L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
        ctx.fini()
        assert pa.read_int(info) == 0
        return np.tril(L)
    finally:
        pa.trsm_inverse_mode(prev, prev_limit)


def _spd(N, cond, seed=3):
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((N, N)))
    S = (q * np.geomspace(1.0, 1.0 / cond, N)) @ q.T
    return 0.5 * (S + S.T)


def test_default_mode_is_auto(pa):
    assert pa.trsm_inverse_mode() == 1
    assert pa.trsm_inverse_limit() == 1e6  # 7x above the largest estimate of the validated sweep (1.5e5)


def _estimates(L, nb):
    out = []
    for k in range(L.shape[0] // nb - 1):  # the panels that have a solve
        t = L[k * nb:(k + 1) * nb, k * nb:(k + 1) * nb]
        out.append(np.abs(t).max() * np.abs(np.linalg.inv(t)).max())
    return np.array(out)


@pytest.mark.parametrize("cond", [1e2, 1e6, 1e12])
def test_modes_agree_and_auto_switches(pa, cond):
    N, nb = 96, 32
    S = _spd(N, cond)
    L0 = _run(pa, S, N, nb, 0)          # through the inverse
    L2 = _run(pa, S, N, nb, 2)          # substitution
    L1 = _run(pa, S, N, nb, 1)          # auto, default limit
    L1s = _run(pa, S, N, nb, 1, 1.0)    # auto with a limit every panel exceeds
    nS = np.linalg.norm(S)
    for L in (L0, L1, L2, L1s):
        assert np.linalg.norm(L @ L.T - S) / nS < 1e-14
    est = _estimates(L2, nb)
    if (est < pa.trsm_inverse_limit()).all():
        assert np.array_equal(L1, L0)   # every panel below the limit: the inverse path, bit for bit
    if (est > pa.trsm_inverse_limit()).all():
        assert np.array_equal(L1, L2)   # every panel above it: substitution, bit for bit
    assert np.array_equal(L1s, L2)      # limit 1: substitution everywhere
    assert np.linalg.norm(L0 - L2) / np.linalg.norm(L2) < cond * 1e-15
