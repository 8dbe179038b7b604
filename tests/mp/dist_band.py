"""Worker for multi-process tests: diag_band_to_rect.jdf with the source band and
the target row on different ranks (the band_src tasks forward source tiles to
the owners of the target tiles)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(rank, size, job, nb, NT, pad):
    import parsec_amd as pa

    pa.mca_set("device_hip_enabled", "0")
    assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    N = nb * NT
    S = np.random.default_rng(11).standard_normal((N, N))
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=size, Q=1)
    for m in range(A.mt):
        for n in range(A.nt):
            if A.rank_of([m, n]) == rank:
                A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                A.mark_host_modified(m, n)
    ncols = (NT + pad) * (nb + 2)
    B = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb + 1, nb + 2, nb + 1, ncols, P=1, Q=size)
    for n in range(B.nt):
        if B.rank_of([0, n]) == rank:
            B.tile(0, n)[:, :] = 7.0
            B.mark_host_modified(0, n)
    tp = pa.diag_band_to_rect_new(A, B, NT, NT, nb, nb)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    bad = 0
    for k in range(B.nt):
        if B.rank_of([0, k]) != rank:
            continue
        got = np.asarray(B.tile(0, k))
        want = np.zeros((nb + 1, nb + 2))
        if k < NT:
            for j in range(nb):
                col = k * nb + j
                for i in range(nb + 1):
                    r = col + i
                    if r < N and (k < NT - 1 or r // nb == k):
                        want[i, j] = S[r, col]
        if not np.array_equal(got, want):
            bad += 1
            print(f"[{rank}] tile {k} differs", got, want)
    ctx.fini()
    print(f"[{rank}] band ok" if bad == 0 else f"[{rank}] band FAILED")
    return 1 if bad else 0


if __name__ == "__main__":
    r, n, job = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    sys.exit(main(r, n, job, int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])))
