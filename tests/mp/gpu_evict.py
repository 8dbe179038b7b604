"""Worker: DPOTRF on HOST-resident tiles through the GPU tile cache capped at a
fraction of the matrix (device_hip_memory_max), so tiles are evicted and dirty
ones written back asynchronously (W2R) during the factorization; optional
PREFETCH advice on every tile first. Prints stats, exits 0 when correct.

argv: N nb cache_fraction prefetch(0/1)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    N, nb, frac, pref = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    import torch

    torch.cuda.set_device(0)
    import parsec_amd as pa

    pa.require_native()
    pa.mca_set("device_hip_memory_max", str(int(frac * N * N * 8)))
    ctx = pa.init(4)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)  # host storage
    rng = np.random.default_rng(4)
    if N <= 8192:
        R = rng.standard_normal((N, N))
        S = R @ R.T / N + np.eye(N)
    else:  # large N: random symmetric + N I (no O(N^3) host product)
        S = rng.random((N, N)) - 0.5
        S = (S + S.T) * 0.5 + N * np.eye(N)
    NT = N // nb
    for m in range(NT):
        for n in range(NT):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
    gpu = pa.first_gpu_device_index()
    if pref:
        for m in range(NT):
            for n in range(m + 1):
                assert pa.data_advise(A, m, n, gpu, pa.DATA_ADVICE_PREFETCH) == 0
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    st = [d for d in pa.devices() if d["index"] == gpu][0]
    L = np.zeros((N, N))
    for m in range(NT):
        for n in range(m + 1):
            L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
    L = np.tril(L)
    ctx.fini()
    if N <= 8192:
        res = np.linalg.norm(L @ L.T - S) / np.linalg.norm(S)
    else:  # backward error on random vectors: ||S x - L L^T x|| / (||S|| ||x||)
        X = rng.random((N, 4)) - 0.5
        res = np.linalg.norm(S @ X - L @ (L.T @ X)) / (np.linalg.norm(S) * np.linalg.norm(X))
    print(f"evict N={N} nb={nb} cache={frac:.2f} prefetch={pref} info={pa.read_int(info)} residual={res:.3e} "
          f"gpu_tasks={st['executed_tasks']} faults={st['data_faults']} w2r={st['w2r_tasks']} prefetches={st['prefetches']} "
          f"in={st['bytes_in'] >> 20}MiB out={st['bytes_out'] >> 20}MiB", flush=True)
    ok = pa.read_int(info) == 0 and res < 1e-13 and st["executed_tasks"] > 0
    if frac < 1:
        ok = ok and st["data_faults"] > 0 and st["w2r_tasks"] > 0
    if pref:
        ok = ok and st["prefetches"] > 0
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
