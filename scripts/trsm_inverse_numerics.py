"""Numerics of the panel solve through the explicit inverse (dpotrf_L.jdf TRSM:
B := B W^T with W = L(k,k)^-1 from POTRF) against the substitution solve
(blocked TRSM, PARSEC_DPOTRF_TRSM=blocked), on SPD matrices of prescribed
condition number.

Both variants are replayed tile by tile in float64 with numpy (the same DAG and
the same inverse-by-forward-substitution as the CPU bodies; the GPU kernels use
IEEE fp64 FMA in a different summation order, so the error ORDERS carry over;
tests/test_dpotrf_gpu.py::test_trsm_inverse_vs_blocked_gpu checks the GPU
points). Printed per (cond, nb):
  bwd  = ||A - L L^T||_F / ||A||_F            (backward error of the factor)
  L diff = ||L_inv - L_blk||_F / ||L_blk||_F  (the two factors)
  estimate = max over tiles of max|L(k,k)| * max|L(k,k)^-1| (the auto switch)
  solv = ||A x - b|| / (||A|| ||x||)           (solve with the factor)
usage: python scripts/trsm_inverse_numerics.py [--n 2048] [--nb 512 1024]
       [--cond 1e2 1e4 1e6 1e8 1e10 1e12]
"""
import argparse

import numpy as np


def spd_with_cond(n, cond, seed=0, graded=False, nb=None):
    """A = Q diag(s) Q^T, s geometric from 1 to 1/cond. graded=True also applies
    a diagonal scaling D A D with D geometric over [1, cond^(1/4)] -- the case
    where individual diagonal tiles are themselves ill-conditioned. graded="tile":
    A = L0 L0^T with L0 unit-random lower and a diagonal that sweeps
    [1, cond^-1/2] inside EVERY nb-tile, so every L(k,k) has cond ~ cond(A)^1/2
    (the adversarial case for the explicit inverse)."""
    rng = np.random.default_rng(seed)
    if graded == "kahan":
        # every diagonal tile's factor is a (transposed) Kahan triangle
        # diag(1, s, s^2..) (I - c * strictly lower ones): ill-conditioned by its
        # off-diagonal structure, NOT visible in the diagonal ratio; c is set so
        # that cond(L(k,k)) ~ cond(A)^1/2
        target = cond ** 0.5

        def kahan(c):
            sdiag = np.sqrt(1.0 - c * c)
            K = np.tril(-c * np.ones((nb, nb)), -1) + np.eye(nb)
            return sdiag ** np.arange(nb)[:, None] * K

        lo, hi = 0.0, 0.5
        for _ in range(60):
            mid = 0.5 * (lo + hi)
            lo, hi = (mid, hi) if np.linalg.cond(kahan(mid)) < target else (lo, mid)
        K = kahan(lo)
        L0 = np.zeros((n, n))
        for t in range(n // nb):
            L0[t * nb:(t + 1) * nb, t * nb:(t + 1) * nb] = K
        L0 += np.tril(rng.standard_normal((n, n)) * (1e-3 / np.sqrt(n)), -nb)  # weak coupling below the tile diagonal
        return L0 @ L0.T
    if graded == "tile":
        # L0 = D (I + E), E strictly lower and small: cond(L0) ~ cond(D) (an
        # unscaled random triangle would be exponentially ill-conditioned)
        E = np.tril(rng.standard_normal((n, n)) * (0.5 / np.sqrt(n)), -1)
        d = np.tile(np.geomspace(1.0, cond ** -0.5, nb), n // nb)
        L0 = d[:, None] * (np.eye(n) + E)
        return L0 @ L0.T
    q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    s = np.geomspace(1.0, 1.0 / cond, n)
    a = (q * s) @ q.T
    a = 0.5 * (a + a.T)
    if graded:
        d = np.geomspace(1.0, cond ** 0.25, n)
        rng.shuffle(d)
        a = a * d[:, None] * d[None, :]
    return a


def lower_inverse(L):
    # forward substitution on the identity, column by column (jdf_cpu_lower_inverse)
    import scipy.linalg as sl

    return np.tril(sl.solve_triangular(L, np.eye(L.shape[0]), lower=True))


def tiled_cholesky(A, nb, mode):
    """mode 'inverse': TRSM as B W^T (W = L_kk^-1); 'blocked': substitution."""
    import scipy.linalg as sl

    A = A.copy()
    n = A.shape[0]
    NT = n // nb
    T = lambda i, j: (slice(i * nb, (i + 1) * nb), slice(j * nb, (j + 1) * nb))
    for k in range(NT):
        Lkk = np.linalg.cholesky(A[T(k, k)])
        A[T(k, k)] = Lkk
        W = lower_inverse(Lkk) if mode == "inverse" else None
        for m in range(k + 1, NT):
            B = A[T(m, k)]
            A[T(m, k)] = B @ W.T if mode == "inverse" else sl.solve_triangular(Lkk, B.T, lower=True).T
        for m in range(k + 1, NT):
            for j in range(k + 1, m + 1):
                A[T(m, j)] -= A[T(m, k)] @ A[T(j, k)].T
    return np.tril(A)


def metrics(A, L, Lref):
    nA = np.linalg.norm(A)
    bwd = np.linalg.norm(A - L @ L.T) / nA
    fwd = np.linalg.norm(L - Lref) / np.linalg.norm(Lref)
    rng = np.random.default_rng(1)
    x = rng.standard_normal(A.shape[0])
    b = A @ x
    import scipy.linalg as sl

    y = sl.solve_triangular(L, b, lower=True)
    xs = sl.solve_triangular(L.T, y, lower=False)
    solv = np.linalg.norm(A @ xs - b) / (np.linalg.norm(A, 2) * np.linalg.norm(xs))
    return bwd, fwd, solv


def sweep(n, nbs, conds, graded):
    rows = []
    for cond in conds:
        A = None if graded in ("tile", "kahan") else spd_with_cond(n, cond, graded=graded)
        for nb in nbs:
            if graded in ("tile", "kahan"):
                A = spd_with_cond(n, cond, graded=graded, nb=nb)
            Lb = tiled_cholesky(A, nb, "blocked")
            Li = tiled_cholesky(A, nb, "inverse")
            rb, ri = metrics(A, Lb, Lb), metrics(A, Li, Lb)
            kdiag = max(np.linalg.cond(Lb[i * nb:(i + 1) * nb, i * nb:(i + 1) * nb]) for i in range(n // nb))
            # the runtime's on-device estimate: max |l_ii| / min |l_ii| per tile
            # the runtime's on-device estimate (PARSEC_DPOTRF_TRSM=auto): max |L(k,k)| * max |W|,
            # W = L(k,k)^-1, elementwise, per tile
            tiles = [Lb[i * nb:(i + 1) * nb, i * nb:(i + 1) * nb] for i in range(n // nb)]
            dr = max(np.abs(t).max() * np.abs(lower_inverse(t)).max() for t in tiles)
            rows.append((cond, nb, kdiag, dr, rb, ri))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--nb", type=int, nargs="+", default=[512, 1024])
    ap.add_argument("--cond", type=float, nargs="+", default=[1e2, 1e4, 1e6, 1e8, 1e10, 1e12])
    ap.add_argument("--family", nargs="+", default=["plain", "graded", "tile"])
    a = ap.parse_args()
    names = {False: "Q diag(s) Q^T", True: "graded D A D", "tile": "L0 L0^T, diagonal of L0 swept inside every tile",
             "kahan": "L0 L0^T, every diagonal tile of L0 a Kahan triangle (ill-conditioned by structure, not by its diagonal)"}
    fam = {"plain": False, "graded": True, "tile": "tile", "kahan": "kahan"}
    for graded in [fam[f] for f in a.family]:
        print(f"-- n={a.n} {names[graded]}")
        print(f"{'cond(A)':>8} {'nb':>5} {'max cond(Lkk)':>13} {'estimate':>10} | {'bwd blk':>9} {'bwd inv':>9} | {'L diff':>9} | {'solv blk':>9} {'solv inv':>9}")
        for cond, nb, kd, dr, rb, ri in sweep(a.n, a.nb, a.cond, graded):
            print(f"{cond:8.0e} {nb:5d} {kd:13.2e} {dr:10.2e} | {rb[0]:9.2e} {ri[0]:9.2e} | {ri[1]:9.2e} | {rb[2]:9.2e} {ri[2]:9.2e}")


if __name__ == "__main__":
    main()
