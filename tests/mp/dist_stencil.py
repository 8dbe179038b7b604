"""Worker: one rank of the distributed DTD 3D stencil; checks its own blocks
against a numpy sweep of the whole grid. argv: rank size job nx ny nz b iters"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import parsec_amd as pa  # noqa: E402


def main():
    rank, size, job = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    nx, ny, nz, b, iters = (int(x) for x in sys.argv[4:9])
    assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    G = pa.StencilGrid(rank, size, nx, ny, nz, b, b, b)
    _, _, par = pa.stencil3d_run(ctx, G, iters, 0.4, 0.1, False)
    x, y, z = np.arange(nx), np.arange(ny), np.arange(nz)
    f = lambda v, n: (v + 1) / (n + 1) * (1 - (v + 1) / (n + 1))  # noqa: E731
    U = 64.0 * f(z, nz)[:, None, None] * f(y, ny)[None, :, None] * f(x, nx)[None, None, :]
    for _ in range(iters):
        P = np.pad(U, 1)
        U = 0.4 * U + 0.1 * (P[1:-1, 1:-1, :-2] + P[1:-1, 1:-1, 2:] + P[1:-1, :-2, 1:-1] + P[1:-1, 2:, 1:-1] + P[:-2, 1:-1, 1:-1] + P[2:, 1:-1, 1:-1])
    nbx, nby = (nx + b - 1) // b, (ny + b - 1) // b
    err, mine = 0.0, 0
    for blk in range(G.nblocks):
        if G.block_rank(blk) != rank:
            continue
        mine += 1
        ib, jb, kb = blk % nbx, (blk // nbx) % nby, blk // (nbx * nby)
        got = G.block(blk, par)
        ref = U[kb * b:kb * b + got.shape[0], jb * b:jb * b + got.shape[1], ib * b:ib * b + got.shape[2]]
        err = max(err, float(np.abs(got - ref).max()))
    ctx.fini()
    pa.comm_fini()
    print(f"rank {rank} blocks {mine} err {err}")
    sys.exit(0 if err < 1e-12 else 1)


if __name__ == "__main__":
    main()
