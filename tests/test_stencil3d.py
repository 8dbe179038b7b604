"""DTD 3D 7-point stencil (BASELINE.json config 5): numpy-checked on CPU for
regular and ragged block decompositions, distributed over 2 and 3 ranks
(halo faces exchanged between ranks), and on the GPU (gpu marker)."""
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _reference(nx, ny, nz, iters):
    f = lambda v, n: (v + 1) / (n + 1) * (1 - (v + 1) / (n + 1))  # noqa: E731
    U = 64.0 * f(np.arange(nz), nz)[:, None, None] * f(np.arange(ny), ny)[None, :, None] * f(np.arange(nx), nx)[None, None, :]
    for _ in range(iters):
        P = np.pad(U, 1)
        U = 0.4 * U + 0.1 * (P[1:-1, 1:-1, :-2] + P[1:-1, 1:-1, 2:] + P[1:-1, :-2, 1:-1] + P[1:-1, 2:, 1:-1] + P[:-2, 1:-1, 1:-1] + P[2:, 1:-1, 1:-1])
    return U


def _check(pa, G, U, par, b, nx, ny):
    nbx, nby = (nx + b - 1) // b, (ny + b - 1) // b
    err = 0.0
    for blk in range(G.nblocks):
        ib, jb, kb = blk % nbx, (blk // nbx) % nby, blk // (nbx * nby)
        got = G.block(blk, par)
        ref = U[kb * b:kb * b + got.shape[0], jb * b:jb * b + got.shape[1], ib * b:ib * b + got.shape[2]]
        err = max(err, float(np.abs(got - ref).max()))
    return err


@pytest.mark.parametrize("nx,ny,nz,b,iters", [(16, 16, 16, 8, 4), (20, 18, 22, 8, 5), (12, 12, 12, 12, 3)])
def test_stencil_cpu(pa, nx, ny, nz, b, iters):
    ctx = pa.init(4)
    G = pa.StencilGrid(0, 1, nx, ny, nz, b, b, b)
    _, pts, par = pa.stencil3d_run(ctx, G, iters, 0.4, 0.1, False)
    assert pts == nx * ny * nz * iters
    assert _check(pa, G, _reference(nx, ny, nz, iters), par, b, nx, ny) < 1e-13
    ctx.fini()


@pytest.mark.parametrize("nranks", [2, 3])
def test_stencil_distributed(pa, nranks):
    job = "st" + uuid.uuid4().hex[:10]
    env = dict(os.environ, PARSEC_MCA_device_hip_enabled="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp", "dist_stencil.py"), str(r), str(nranks), job, "18", "16", "20", "6", "4"],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env) for r in range(nranks)]
    try:
        for p in procs:
            out, _ = p.communicate(timeout=120)
            assert p.returncode == 0, out
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


@pytest.mark.gpu
@pytest.mark.parametrize("n,b,iters", [(96, 32, 6), (130, 64, 4), (99, 33, 3), (300, 256, 3)])
def test_stencil_gpu(pa, n, b, iters):
    ctx = pa.init(4)
    dev = pa.first_gpu_device_index()
    if dev < 0:
        pytest.skip("no GPU")
    G = pa.StencilGrid(0, 1, n, n, n, b, b, b, device=dev)
    _, _, par = pa.stencil3d_run(ctx, G, iters, 0.4, 0.1, True)
    assert _check(pa, G, _reference(n, n, n, iters), par, b, n, n) < 1e-12
    devs = [d for d in pa.devices() if d["type"] == pa.DEV_HIP]
    assert devs and devs[0]["executed_tasks"] > 0
    ctx.fini()
