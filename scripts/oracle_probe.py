"""Root-cause probe for the round-2 shared-GPU oracle anomaly: torch.linalg.cholesky
on the GPU disagreed with host LAPACK by ~2e-3 in 2 of 4 processes sharing one
MI355X while the runtime was loaded. This runs the same oracle with the runtime
absent / imported / initialised (+ one DPOTRF), in N concurrent processes.

    python scripts/oracle_probe.py --procs 4 --mode none
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode, n, idx):
    import numpy as np
    import scipy.linalg
    import torch

    if mode != "none":
        sys.path.insert(0, ROOT)
        import parsec_amd as pa
    torch.cuda.set_device(0)
    g = torch.Generator().manual_seed(123)
    R = torch.rand((n, n), dtype=torch.float64, generator=g)
    S = (R + R.t()) / 2 + n * torch.eye(n, dtype=torch.float64)
    Lh = scipy.linalg.cholesky(S.numpy(), lower=True)
    if mode == "init":
        ctx = pa.init(2)
        gpu = pa.first_gpu_device_index()
        nb = 512
        NT = n // nb
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
        store.copy_(S.cuda().reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, n, n, device=gpu, ptr=store.data_ptr())
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        torch.cuda.synchronize()
    res = []
    for rep in range(3):
        Lg = torch.linalg.cholesky(S.cuda()).cpu().numpy()
        res.append(float(np.abs(Lg - Lh).max() / np.abs(Lh).max()))
    if mode == "init":
        ctx.fini()
    print(f"proc {idx} mode {mode} torch GPU cholesky vs host (3 reps): " + " ".join(f"{r:.3e}" for r in res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--mode", choices=["none", "import", "init"], default="none")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--child", type=int, default=-1)
    a = ap.parse_args()
    if a.child >= 0:
        child(a.mode, a.n, a.child)
        return
    ps = [subprocess.Popen([sys.executable, __file__, "--mode", a.mode, "--n", str(a.n), "--child", str(i)]) for i in range(a.procs)]
    rc = max(p.wait() for p in ps)
    sys.exit(rc)


if __name__ == "__main__":
    main()
