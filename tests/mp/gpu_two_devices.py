"""Worker: DPOTRF on HOST-resident tiles with the GPU registered as two devices
(device_hip_replicas 2): the engine spreads the GPU tasks over both, so tiles
written on one device are read on the other (device-to-device stage-in, and
read-only inputs staged from the other device's copy: device_hip_peer_stage_in).
Optionally with the tile cache capped (eviction + write-back on both devices).
Prints per-device stats, exits 0 when the factor is correct and both devices
worked and exchanged tiles.

argv: N nb cache_fraction(0 = uncapped)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    N, nb, frac = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    import torch

    torch.cuda.set_device(0)
    import parsec_amd as pa

    pa.require_native()
    pa.mca_set("device_hip_replicas", "2")
    if frac > 0:
        pa.mca_set("device_hip_memory_max", str(int(frac * N * N * 8)))
    ctx = pa.init(4)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)  # host storage
    rng = np.random.default_rng(7)
    R = rng.standard_normal((N, N))
    S = R @ R.T / N + np.eye(N)
    NT = N // nb
    for m in range(NT):
        for n in range(NT):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    gpus = [d for d in pa.devices() if d["name"].startswith("hip")]
    L = np.zeros((N, N))
    for m in range(NT):
        for n in range(m + 1):
            L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
    L = np.tril(L)
    ctx.fini()
    res = np.linalg.norm(L @ L.T - S) / np.linalg.norm(S)
    per = " ".join(f"{d['name']}:tasks={d['executed_tasks']},d2d={d['bytes_d2d'] >> 20}MiB,in={d['bytes_in'] >> 20}MiB,faults={d['data_faults']}" for d in gpus)
    print(f"two_devices N={N} nb={nb} cache={frac:.2f} info={pa.read_int(info)} residual={res:.3e} {per}", flush=True)
    ok = pa.read_int(info) == 0 and res < 1e-13 and len(gpus) == 2
    ok = ok and all(d["executed_tasks"] > 0 for d in gpus) and sum(d["bytes_d2d"] for d in gpus) > 0
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
