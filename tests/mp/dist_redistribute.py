"""Worker: one rank of a distributed redistribution (reference
tests/collections/redistribute/testing_redistribute.c, re-specified). The
source is a P x Q block-cyclic matrix with smb x snb tiles, the target a Q x P
one with dmb x dnb tiles; a window of the source moves to another offset of
the target. Every element of the source holds its global position, so each
rank checks its own target tiles exactly: window cells must hold the source
position they map from, every other cell keeps its fill value.
argv: rank size job method smb snb dmb dnb size_row size_col disi_s disj_s disi_t disj_t"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import parsec_amd as pa  # noqa: E402

SM, SN, TM, TN = 70, 64, 66, 72   # source / target matrix sizes


def grid(size):
    p = int(size ** 0.5)
    while size % p:
        p -= 1
    return p, size // p


def main():
    rank, size, job, method = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    smb, snb, dmb, dnb, sr, sc, si, sj, ti, tj = map(int, sys.argv[5:15])
    if size > 1:
        assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    P, Q = grid(size)
    S = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, smb, snb, SM, SN, P=P, Q=Q)
    T = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, dmb, dnb, TM, TN, P=Q, Q=P)
    for m in range(S.mt):
        for n in range(S.nt):
            if S.rank_of([m, n]) != rank:
                continue
            t = S.tile(m, n)
            ii, jj = np.meshgrid(np.arange(m * smb, m * smb + t.shape[0]), np.arange(n * snb, n * snb + t.shape[1]), indexing="ij")
            t[:, :] = ii * 1000.0 + jj
    for m in range(T.mt):
        for n in range(T.nt):
            if T.rank_of([m, n]) == rank:
                T.tile(m, n)[:, :] = -1.0
    rc = pa.redistribute(ctx, S, T, sr, sc, si, sj, ti, tj, method=method)
    assert rc == 0, rc
    bad = 0
    checked = 0
    for m in range(T.mt):
        for n in range(T.nt):
            if T.rank_of([m, n]) != rank:
                continue
            t = T.tile(m, n)
            for r in range(t.shape[0]):
                for c in range(t.shape[1]):
                    gi, gj = m * dmb + r, n * dnb + c
                    if ti <= gi < ti + sr and tj <= gj < tj + sc:
                        want = (gi - ti + si) * 1000.0 + (gj - tj + sj)
                        checked += 1
                    else:
                        want = -1.0
                    if t[r, c] != want:
                        bad += 1
    ctx.fini()
    if size > 1:
        pa.comm_fini()
    print(f"rank {rank} method {method} checked {checked} bad {bad}")
    sys.exit(0 if bad == 0 else 1)


if __name__ == "__main__":
    main()
