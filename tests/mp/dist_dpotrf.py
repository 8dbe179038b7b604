"""Worker for multi-process tests: distributed PTG DPOTRF on host tiles (CPU bodies)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(rank, size, job, N, nb, P, Q, sched="lfq", topo="star", termdet="local"):
    import parsec_amd as pa

    pa.mca_set("device_hip_enabled", "0")
    pa.mca_set("mca_sched", sched)
    pa.mca_set("runtime_comm_coll_bcast", topo)
    assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=P, Q=Q)
    rng = np.random.default_rng(7)
    R = rng.standard_normal((N, N))
    S = (R + R.T) / 2 + N * np.eye(N)
    for m in range(A.mt):
        for n in range(A.nt):
            if A.rank_of([m, n]) == rank:
                A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                A.mark_host_modified(m, n)
    if os.environ.get("DPOTRF_TASKPOOL") == "jdf":
        tp, info = pa.dpotrf_jdf_new(A)  # ptgpp-compiled algos/jdf/dpotrf_L.jdf
    else:
        tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    tp.termdet = termdet
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    # check the local tiles of L against numpy's factor
    Lref = np.linalg.cholesky(S)
    err = 0.0
    for m in range(A.mt):
        for n in range(m + 1):
            if A.rank_of([m, n]) == rank:
                t = A.tile(m, n)
                ref = Lref[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                if m == n:
                    t, ref = np.tril(t), np.tril(ref)
                err = max(err, float(np.abs(t - ref).max()))
    if os.environ.get("DIST_PRINT_COMM_STATS"):
        st = pa.comm_stats()
        print("comm_stats " + " ".join(f"{k}={v}" for k, v in sorted(st.items())), flush=True)
    ctx.fini()
    pa.comm_fini()
    return err, pa.read_int(info)


if __name__ == "__main__":
    r, s = int(sys.argv[1]), int(sys.argv[2])
    err, info = main(r, s, sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7]),
                     *(sys.argv[8:]))
    print(f"rank {r} err {err:.3e} info {info}", flush=True)
    sys.exit(0 if err < 1e-10 and info == 0 else 1)
