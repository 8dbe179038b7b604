"""Worker: one rank of a distributed PTG DGEQRF on host tiles (CPU bodies),
2D block-cyclic P x Q; writes this rank's tiles of R (zeros elsewhere).
argv: rank size job M N nb P Q outdir [hqr_domain]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import parsec_amd as pa  # noqa: E402


def main():
    rank, size, job = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    M, N, nb, P, Q = (int(x) for x in sys.argv[4:9])
    outdir = sys.argv[9]
    pa.mca_set("device_hip_enabled", "0")
    assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, M, N, P=P, Q=Q)
    T = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, M, N, P=P, Q=Q)
    S = np.random.default_rng(5).standard_normal((M, N))
    for m in range(A.mt):
        for n in range(A.nt):
            if A.rank_of([m, n]) == rank:
                blk = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                A.tile(m, n)[:blk.shape[0], :blk.shape[1]] = blk
                A.mark_host_modified(m, n)
    if len(sys.argv) > 10 and int(sys.argv[10]) > 0:  # hierarchical tree, TS domains of argv[10] rows
        TT = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, M, N, P=P, Q=Q)
        tp = pa.dgeqrf_hqr_new(A, T, TT, int(sys.argv[10]))
    else:
        tp = (pa.dgeqrf_jdf_new(A, T) if os.environ.get("QR_TASKPOOL", "jdf") == "jdf" else pa.dgeqrf_new(A, T, 32))
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    R = np.zeros((M, N))
    for m in range(A.mt):
        for n in range(A.nt):
            if A.rank_of([m, n]) == rank:
                blk = R[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                blk[:, :] = A.tile(m, n)[:blk.shape[0], :blk.shape[1]]
    R = np.triu(R)[:min(M, N)]
    ctx.fini()
    pa.comm_fini()
    np.save(os.path.join(outdir, f"R{rank}.npy"), R)  # zero outside this rank's tiles
    print(f"rank {rank} done")


if __name__ == "__main__":
    main()
