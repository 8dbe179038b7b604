#!/usr/bin/env python3
"""The other BASELINE.json workloads, one JSON line each (rank 0):

  qr       tiled Householder QR (PTG DGEQRF: GEQRT/UNMQR/TSQRT/TSMQR), matrix and
           T factors resident in HBM, GFLOP/s with 4/3 N^3 (config 4)
  stencil  DTD 3D 7-point Jacobi stencil, halo faces between blocks (and ranks),
           GPU bodies, Gpoint-updates/s and GFLOP/s at 8 flop/point (config 5)
  dtd_gemm DTD tiled DGEMM C += A B on 4 x 4 tiles, CPU bodies in one process
           (config 1, the plumbing check), GFLOP/s

Multi-GPU: launch like bench.py (torch.distributed.run, one rank per GPU).

    python benchmarks/bench_workloads.py qr --n 16384 --nb 512
    python benchmarks/bench_workloads.py stencil --n 512 --b 128 --iters 20
    python benchmarks/bench_workloads.py dtd_gemm --n 2048
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _comm(pa, world, rank, local, gpu=True):
    if world > 1:
        job = "_".join([os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "wl"), str(os.getppid())])
        if pa.comm_init(rank, world, job, local if gpu else -1) != 0:
            raise RuntimeError("comm_init failed")


def bench_qr(args):
    import torch
    import torch.distributed as dist

    world, rank, local = _dist()
    if args.share_gpu:  # validation mode: every rank on GPU 0, collectives over gloo
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import parsec_amd as pa

    pa.require_native()
    pa.mca_set("device_hip_mask", str(1 << local))
    _comm(pa, world, rank, local)
    ctx = pa.init(args.cores)

    def allreduce(v, op=None):  # on the GPU (RCCL) or, sharing one GPU, on host copies (gloo)
        if world == 1:
            return v
        kw = {} if op is None else {"op": op}
        if args.share_gpu:
            c = v.cpu()
            dist.all_reduce(c, **kw)
            v.copy_(c)
        else:
            dist.all_reduce(v, **kw)
        return v
    gpu = pa.first_gpu_device_index()
    N, nb = args.n, args.nb
    # process grid: --qr-grid 1d = P x 1 row-cyclic (the TS chain of a panel
    # crosses every rank), 2d = the most square P x Q (P >= Q), which halves the
    # ranks a panel chain crosses at 8 GPUs and spreads the trailing update
    if args.qr_grid == "2d":
        P = int(world ** 0.5)
        while world % P:
            P -= 1
        P, Q = max(P, world // P), min(P, world // P)
    else:
        P, Q = world, 1
    NT = (N + nb - 1) // nb
    myrow, mycol = rank // Q, rank % Q
    lm = sum(1 for g in range(NT) if g % P == myrow)
    ln = sum(1 for g in range(NT) if g % Q == mycol)
    storeA = torch.empty((ln, lm, nb, nb), dtype=torch.float64, device="cuda")
    storeT = torch.zeros((ln, lm, nb, nb), dtype=torch.float64, device="cuda")
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=P, Q=Q, device=gpu, ptr=storeA.data_ptr())
    T = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=P, Q=Q, device=gpu, ptr=storeT.data_ptr())
    # auto: one process row -> the flat TS tree from the ptgpp-compiled
    # dgeqrf.jdf (what the hierarchical tree reduces to there); several process
    # rows -> the hierarchical tree (TT merges across the rows)
    hqr = args.qr_tree == "hqr" or (args.qr_tree == "auto" and P > 1)
    use_jdf = not hqr and args.taskpool == "jdf"
    if hqr:  # TT-kernel reflectors of the hierarchical tree
        storeTT = torch.zeros((ln, lm, nb, nb), dtype=torch.float64, device="cuda")
        TT = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=P, Q=Q, device=gpu, ptr=storeTT.data_ptr())
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    storeA.copy_(torch.rand(storeA.shape, dtype=torch.float64, device="cuda", generator=g) - 0.5)
    backup = storeA.clone()

    def step():
        storeA.copy_(backup)
        storeT.zero_()
        torch.cuda.synchronize()
        tp = pa.dgeqrf_hqr_new(A, T, TT, args.qr_domain) if hqr else pa.dgeqrf_jdf_new(A, T) if use_jdf else pa.dgeqrf_new(A, T, args.ib)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        barrier()
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = (time.perf_counter() - t0) / args.steps
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        allreduce(tt, dist.ReduceOp.MAX)
        dt = float(tt.item())
    check = None
    if args.check:
        # R of the last timed factorization against the input, outside the timed
        # region. Q orthogonal => A^T A = R^T R; probed with a random x from the
        # local tiles and summed over ranks (4 all-reduces of N-vectors):
        # ||A^T (A x) - R^T (R x)|| / (||A||_F^2 ||x||)
        torch.cuda.synchronize()
        gx = torch.Generator(device="cuda").manual_seed(99)
        x = torch.rand(N, dtype=torch.float64, device="cuda", generator=gx) - 0.5
        At, Rt = backup.view(-1, nb, nb), storeA.view(-1, nb, nb)
        loc = [(m, n, A.local_index(m, n)) for n in range(NT) for m in range(NT)]
        loc = [(m, n, li) for (m, n, li) in loc if li >= 0]

        def allsum(v):
            return allreduce(v)

        def blk(t, m, n):
            return t.t()[:min(nb, N - m * nb), :min(nb, N - n * nb)]

        def sl(i):
            return slice(i * nb, min(N, (i + 1) * nb))

        ax, rx = torch.zeros(N, dtype=torch.float64, device="cuda"), torch.zeros(N, dtype=torch.float64, device="cuda")
        fro = torch.zeros(1, dtype=torch.float64, device="cuda")
        for m, n, li in loc:
            a = blk(At[li], m, n)
            ax[sl(m)] += a @ x[sl(n)]
            fro += (a * a).sum()
            if m <= n:
                r = blk(Rt[li], m, n)
                rx[sl(m)] += (torch.triu(r) if m == n else r) @ x[sl(n)]
        allsum(ax), allsum(rx), allsum(fro)
        ata, rtr = torch.zeros(N, dtype=torch.float64, device="cuda"), torch.zeros(N, dtype=torch.float64, device="cuda")
        for m, n, li in loc:
            ata[sl(n)] += blk(At[li], m, n).t() @ ax[sl(m)]
            if m <= n:
                r = blk(Rt[li], m, n)
                rtr[sl(n)] += (torch.triu(r) if m == n else r).t() @ rx[sl(m)]
        allsum(ata), allsum(rtr)
        check = float(torch.linalg.norm(ata - rtr) / (fro.item() * torch.linalg.norm(x)))
    ctx.fini()
    if world > 1:
        pa.comm_fini()
    out = {"metric": "GFLOP/s tiled DGEQRF (PTG, HBM-resident)", "value": round(4.0 / 3.0 * N ** 3 / dt / 1e9, 1), "unit": "GFLOP/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
           "dtype": "fp64", "data": "synthetic uniform(-0.5, 0.5)", "config": {"model": "tiled DGEQRF (" + ((f"hierarchical, TS domains of {args.qr_domain}" if args.qr_domain > 0 else "hierarchical, flat TS per process row") + ", TT binary trees" if hqr else "flat TS tree") + (", ptgpp-compiled dgeqrf.jdf" if use_jdf else ", hand-built C++ DAG") + ")", "N": N, "nb": nb, "ib": 32,
                                                                             "parallelism": f"2D block-cyclic P{P}xQ{Q}" if Q > 1 else f"1D row-cyclic P{P}x1"}}
    if check is not None:
        out["residual_AtAx_vs_RtRx"] = check
    if args.share_gpu:
        out["note"] = "validation mode: all ranks share GPU 0; not a scaling measurement"
    if world > 1:
        dist.destroy_process_group()
    return out, rank


def bench_stencil(args):
    world, rank, local = _dist()
    import torch

    dev = 0 if args.share_gpu else local  # --share-gpu: every rank on GPU 0 (halo-path validation, not scaling)
    torch.cuda.set_device(dev)
    import parsec_amd as pa

    pa.require_native()
    pa.mca_set("device_hip_mask", str(1 << dev))
    _comm(pa, world, rank, dev)
    ctx = pa.init(args.cores)
    # grid resident in HBM (the home device of every block and face buffer)
    G = pa.StencilGrid(rank, world, args.n, args.n, args.n, args.b, args.b, args.b, device=pa.first_gpu_device_index())
    pa.stencil3d_run(ctx, G, 2, 0.4, 0.1, True)  # warmup: tiles to HBM, kernels loaded
    secs, pts, _ = pa.stencil3d_run(ctx, G, args.iters, 0.4, 0.1, True)
    if world > 1:
        secs = pa.comm_allreduce_max_f64(secs) if hasattr(pa, "comm_allreduce_max_f64") else secs
    ctx.fini()
    if world > 1:
        pa.comm_fini()
    gpts = pts / secs / 1e9
    out = {"metric": "Gpoint-updates/s DTD 3D 7-point stencil", "value": round(gpts, 2), "unit": "Gpoints/s", "gflops": round(8 * gpts, 1),
           "n_gpus": world, "steps": args.iters, "ms_per_step": round(secs / args.iters * 1e3, 3), "higher_is_better": True, "dtype": "fp64",
           "data": "synthetic smooth field", "config": {"model": "DTD stencil3d", "grid": [args.n] * 3, "block": args.b, "ranks": world}}
    if args.share_gpu:
        out["note"] = f"validation mode: all {world} ranks share GPU 0 (halo faces cross ranks over IPC); not a scaling measurement"
    return out, rank


def bench_dtd_gemm(args):
    import numpy as np

    import parsec_amd as pa

    pa.mca_set("device_hip_enabled", "0")
    ctx = pa.init(args.cores)
    N, nt = args.n, 4
    nb = N // nt
    mats = [pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N) for _ in range(3)]
    rng = np.random.default_rng(0)
    for M in mats:
        for m in range(nt):
            for n in range(nt):
                M.tile(m, n)[:, :] = rng.standard_normal((nb, nb))
    pa.dtd_dgemm(ctx, 1.0, mats[0], mats[1], 1.0, mats[2], False)  # warmup
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pa.dtd_dgemm(ctx, 1.0, mats[0], mats[1], 1.0, mats[2], False)
    dt = (time.perf_counter() - t0) / args.steps
    ctx.fini()
    out = {"metric": "GFLOP/s DTD tiled DGEMM (CPU bodies, 1 process)", "value": round(2.0 * N ** 3 / dt / 1e9, 2), "unit": "GFLOP/s",
           "n_gpus": 0, "steps": args.steps, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "fp64",
           "config": {"model": "DTD dgemm", "N": N, "tiles": "4x4", "cores": args.cores}}
    return out, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["qr", "stencil", "dtd_gemm"])
    ap.add_argument("--n", "--size", dest="n", type=int, default=None, help="matrix order (use --size under torchrun)")
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--ib", type=int, default=32, help="qr: accepted for the reference's command line; both taskpools factor 32-column sub-panels (qr_sub2c) and apply one nb x nb block reflector per tile")
    ap.add_argument("--b", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cores", type=int, default=4)
    ap.add_argument("--qr-grid", choices=["1d", "2d"], default="2d", help="qr: process grid over the ranks")
    ap.add_argument("--share-gpu", action="store_true", help="qr / stencil: validation mode, every rank on GPU 0; not a scaling measurement")
    ap.add_argument("--check", action="store_true", help="qr: verify R (||A^T A x - R^T R x|| / (||A||_F^2 ||x||), all ranks) after the timed steps")
    ap.add_argument("--qr-tree", choices=["auto", "hqr", "flat"], default="auto", help="qr: hierarchical (TS domains + TT trees), flat TS tree, or auto (flat on one process row, hierarchical otherwise)")
    ap.add_argument("--taskpool", choices=["jdf", "ir"], default="jdf", help="qr flat tree: the ptgpp-compiled dgeqrf.jdf (default) or the hand-built C++ DAG (dgeqrf.cpp)")
    ap.add_argument("--qr-domain", type=int, default=0,
                    help="qr: rows per TS domain of the hierarchical tree (0: one flat TS chain per process row, TT binary tree across process rows; 1 GPU measured fastest flat: profiles/r3_qr_tree_ab.jsonl)")
    args = ap.parse_args()
    if args.n is None:
        args.n = {"qr": 16384, "stencil": 512, "dtd_gemm": 2048}[args.workload]
    fn = {"qr": bench_qr, "stencil": bench_stencil, "dtd_gemm": bench_dtd_gemm}[args.workload]
    out, rank = fn(args)
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
