#!/usr/bin/env python3
"""Headline benchmark: tiled DPOTRF (lower, fp64) on a 2D block-cyclic matrix
resident in HBM, one process per MI355X, PTG taskpool, batched MFMA tile kernels.

Metric (BASELINE.json): GFLOP/s (whole node) tiled DPOTRF 2D block-cyclic at
1/2/4/8 MI355X. The taskpool is the one parsec-ptgpp compiles from
csrc/algos/jdf/dpotrf_L.jdf. Default config = BASELINE config 3 (N=65536, nb=1024), the
same problem at every GPU count (strong scaling). `--n 16384 --nb 512`
reproduces config 2 (1 GPU).

    python bench.py --gpus 1 --steps 3 --warmup 1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 8

Every step restores the input matrix (device copy, inside the timed region),
builds the taskpool and factorizes. Flops = N^3/3 + N^2/2 + N/6.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def grid_of(n):
    p = int(n ** 0.5)
    while n % p:
        p -= 1
    return max(p, n // p), min(p, n // p)  # P >= Q


_T0 = time.time()


def _stage(msg):
    if os.environ.get("PARSEC_BENCH_VERBOSE"):
        print(f"[bench rank {os.environ.get('RANK', '0')} +{time.time() - _T0:.3f}s] {msg}", file=sys.stderr, flush=True)


def residual_probe(torch, dist, world, A, store, backup, nb, N, rank, share_gpu):
    """||A x - L L^T x||_2 / (||A||_F ||x||_2) from the local tiles of A (backup,
    lower half) and L (store); the three partial vectors and ||A||_F^2 are summed
    over ranks (two all-reduces)."""
    dev = store.device
    g = torch.Generator(device=dev).manual_seed(4242)
    x = torch.rand(N, dtype=torch.float64, device=dev, generator=g) - 0.5
    tiles, btiles = store.view(-1, nb, nb), backup.view(-1, nb, nb)
    NT = A.nt
    loc = [(m, n, A.local_index(m, n)) for n in range(NT) for m in range(n, NT)]
    loc = [(m, n, li) for (m, n, li) in loc if li >= 0]

    def blk(t, m, n):  # column-major tile -> (rows x cols) matrix view
        r, c = min(nb, N - m * nb), min(nb, N - n * nb)
        return t.t()[:r, :c]

    def allsum(v):
        if world > 1:
            if share_gpu:
                c = v.cpu()
                dist.all_reduce(c)
                v.copy_(c)
            else:
                dist.all_reduce(v)
        return v

    ax = torch.zeros(N, dtype=torch.float64, device=dev)
    ltx = torch.zeros(N, dtype=torch.float64, device=dev)
    fro = torch.zeros(1, dtype=torch.float64, device=dev)
    for m, n, li in loc:
        a = blk(btiles[li], m, n)
        l = blk(tiles[li], m, n)
        sm, sn = slice(m * nb, m * nb + a.shape[0]), slice(n * nb, n * nb + a.shape[1])
        if m == n:
            a = torch.tril(a) + torch.tril(a, -1).t()
            l = torch.tril(l)
            fro += (a * a).sum()
        else:
            ax[sn] += a.t() @ x[sm]
            fro += 2 * (a * a).sum()
        ax[sm] += a @ x[sn]
        ltx[sn] += l.t() @ x[sm]
    allsum(ltx)
    llx = torch.zeros(N, dtype=torch.float64, device=dev)
    for m, n, li in loc:
        l = blk(tiles[li], m, n)
        if m == n:
            l = torch.tril(l)
        llx[m * nb:m * nb + l.shape[0]] += l @ ltx[n * nb:n * nb + l.shape[1]]
    v = torch.cat([ax - llx, fro])
    allsum(v)
    return float(torch.linalg.norm(v[:N]) / (torch.sqrt(v[N]) * torch.linalg.norm(x)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", "--n", dest="n", type=int, default=65536, help="matrix order N (use --size under torchrun)")
    ap.add_argument("--nb", type=int, default=1024)
    ap.add_argument("--cores", type=int, default=int(os.environ.get("PARSEC_BENCH_CORES", "4")))
    ap.add_argument("--check", action="store_true", help="verify the factorization (small N only)")
    ap.add_argument("--mca", nargs=2, action="append", default=[])
    ap.add_argument("--taskpool", choices=["ir", "jdf"], default="jdf",
                    help="jdf (default): the DAG compiled by parsec-ptgpp from csrc/algos/jdf/dpotrf_L.jdf; ir: the same DAG built by hand in C++ (csrc/algos/dpotrf.cpp, a test fixture)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="validation mode: every rank uses GPU 0 (torch gloo for the bench's own barriers; the runtime's IPC device plane as always)")
    ap.add_argument("--allow-host-plane", action="store_true",
                    help="multi-rank: accept ranks whose device plane fell back to host staging (default: such a run exits non-zero)")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu: host-resident tiles and CPU task bodies, gloo for the bench's own collectives (tests of the distributed path and its reporting on machines without a GPU; not a measurement)")
    args = ap.parse_args()
    cpu = args.device == "cpu"

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    if args.share_gpu:
        local = 0
    tdev = "cpu" if cpu else "cuda"
    coll_dev = "cpu" if (cpu or args.share_gpu) else "cuda"  # device of the bench's own collective tensors
    if not cpu:
        torch.cuda.set_device(local)
    if world > 1:
        if args.share_gpu or cpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    def gather_rows(vals):
        """every rank's row of ints, in rank order (all ranks call it)"""
        mine = torch.tensor(vals, dtype=torch.int64, device=coll_dev)
        if world == 1:
            return [mine.tolist()]
        got = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(got, mine)
        return [g.tolist() for g in got]

    N, nb = args.n, args.nb
    P, Q = grid_of(world)
    base = {
        "metric": "GFLOP/s (whole node) tiled DPOTRF 2D block-cyclic at 1/2/4/8 MI355X",
        "value": None,
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp64",
        "data": "synthetic random symmetric + N*I (DPLASMA plgsy convention), " + ("host-resident tiles" if cpu else "HBM-resident tiles"),
        "config": {"model": "tiled DPOTRF lower (PTG, ptgpp-compiled dpotrf_L.jdf)" if args.taskpool == "jdf" else "tiled DPOTRF lower (PTG, hand-built C++ DAG)", "N": N, "nb": nb, "global_batch": 1, "seq_len": N,
                   "parallelism": f"2D block-cyclic P{P}xQ{Q}, 1 process/GPU", "threads_per_rank": args.cores},
    }
    if cpu:
        base["note"] = "--device cpu: CPU task bodies, host tiles; a test of the distributed path, not a measurement"
    elif args.share_gpu:
        base["note"] = "validation mode: all ranks share GPU 0; not a scaling measurement"

    def fail(code, msg, extra):
        """rank 0 prints the JSON line (what is known so far + the error) BEFORE
        the non-zero exit, so a failed multi-GPU run still reports its route
        tables"""
        if rank == 0:
            out = dict(base, **extra)
            out["error"] = msg
            print(json.dumps(out), flush=True)
            print(f"error: {msg}", file=sys.stderr, flush=True)
        raise SystemExit(code)

    _stage("process group up")
    import parsec_amd as pa

    pa.require_native()
    if not cpu:
        pa.mca_set("device_hip_mask", str(1 << local))
    for k, v in args.mca:
        pa.mca_set(k, v)
    if world > 1:
        # unique per launch: the launcher pid is shared by all ranks of one job
        job = "_".join([os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "bench"), str(os.getppid())])
        rc = pa.comm_init(rank, world, job, -1 if cpu else local)
        if rc != 0:
            raise RuntimeError(f"comm_init failed rc={rc}")
    _stage("comm up")
    # every rank's device plane (ipc: remote tiles move GPU -> GPU over xGMI;
    # host: staged through host memory) and its IPC start-up probe of every peer
    # (bits: 1 open, 2 copy-engine pull, 4 copy kernel, 8 host read; -1 not
    # probed), reported in the JSON line; a multi-rank run on the host plane is
    # not the headline path and fails loudly -- after printing the tables
    planes = [{"rank": 0, "plane": "none", "status": 0}]
    probe = None
    if world > 1:
        code = {"ipc": 1, "host": 0}.get(pa.comm_device_plane(), -1)
        rows = gather_rows([code, pa.comm_plane_status()])
        planes = [{"rank": r, "plane": {1: "ipc", 0: "host"}.get(g[0], "?"), "status": g[1]} for r, g in enumerate(rows)]
        table = pa.comm_probe_table() or [(-1, 0)] * world
        codes = gather_rows([c for c, _ in table])
        tries = gather_rows([a for _, a in table])
        probe = {"codes": codes, "open_attempts": tries}
        if any(p["plane"] != "ipc" for p in planes) and not args.allow_host_plane:
            bad = [(r, q, codes[r][q]) for r in range(world) for q in range(world) if codes[r][q] not in (0,)]
            fail(3, f"device plane is not ipc on every rank (rank, peer, probe bits): {bad[:16]}", {"device_plane": planes, "ipc_probe": probe})
    ctx = pa.init(args.cores)
    _stage("context up")
    gpu = 0 if cpu else pa.first_gpu_device_index()
    if gpu < 0:
        raise RuntimeError("no GPU device registered in the runtime")

    # storage owned by torch so generation / restore are plain torch ops
    NTg = (N + nb - 1) // nb
    llm = sum(1 for g in range(NTg) if g % P == rank // Q)
    lln = sum(1 for g in range(NTg) if g % Q == rank % Q)
    store = torch.empty((lln, llm, nb, nb), dtype=torch.float64, device=tdev)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, nb, nb, N, N, P=P, Q=Q, device=gpu, ptr=store.data_ptr())
    NT = A.nt
    # synthetic SPD input: random symmetric, diagonally dominant (lower tiles only)
    gen = torch.Generator(device=tdev)
    for n in range(NT):
        for m in range(n, NT):
            li = A.local_index(m, n)
            if li < 0:
                continue
            gen.manual_seed(1_000_003 * m + n)
            t = torch.rand((nb, nb), dtype=torch.float64, device=tdev, generator=gen) - 0.5
            if m == n:
                t = (t + t.t()) * 0.5 + N * torch.eye(nb, dtype=torch.float64, device=tdev)
            store.view(-1, nb, nb)[li].copy_(t.t())
    backup = store.clone()
    sync()

    def step():
        store.copy_(backup)
        sync()
        tp, info = pa.dpotrf_jdf_new(A) if args.taskpool == "jdf" else pa.dpotrf_new(A, pa.MATRIX_LOWER)
        ctx.add_taskpool(tp)
        ctx.start()
        _stage("taskpool started")
        ctx.wait()
        _stage("taskpool done")
        return pa.read_int(info)

    def barrier():
        sync()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        barrier()
        if step() != 0:
            raise RuntimeError("dpotrf reported a non-SPD matrix")
    barrier()
    t0 = time.perf_counter()
    bad = 0
    for _ in range(args.steps):
        bad = bad or step()  # LAPACK info of every timed factorization (host int, no sync)
    barrier()
    if bad:
        raise RuntimeError(f"dpotrf info={bad} in a timed step")
    dt = time.perf_counter() - t0
    _stage("timed region done")
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    flops = N ** 3 / 3 + N ** 2 / 2 + N / 6
    gflops = flops / (ms * 1e-3) / 1e9

    # Backward error of the LAST timed factorization over the whole matrix (outside
    # the timed region): r = ||A x - L (L^T x)|| / (||A||_F ||x||) for a random x,
    # each rank contributing its local tiles, partial vectors summed over ranks.
    resid = residual_probe(torch, dist, world, A, store, backup, nb, N, rank, args.share_gpu or cpu)
    _stage(f"residual {resid:.3e}")
    if not resid < 1e-12:
        raise RuntimeError(f"DPOTRF residual {resid:.3e} too large")

    check = None
    if args.check:
        # every rank rebuilds the full input (same seeds), factors it with torch
        # and compares its own tiles of L; the max error is reduced over ranks
        full = torch.zeros((N, N), dtype=torch.float64, device=tdev)
        for n in range(NT):
            for m in range(n, NT):
                gen.manual_seed(1_000_003 * m + n)
                t = torch.rand((nb, nb), dtype=torch.float64, device=tdev, generator=gen) - 0.5
                if m == n:
                    t = (t + t.t()) * 0.5 + N * torch.eye(nb, dtype=torch.float64, device=tdev)
                full[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = t
        S = torch.tril(full) + torch.tril(full, -1).t()
        # host LAPACK reference: torch's GPU Cholesky is intermittently wrong when
        # several processes share the GPU, with or without this runtime loaded
        # (profiles/r3_oracle_root_cause.txt)
        Lref = torch.linalg.cholesky(S.cpu()).to(S.device)
        err = 0.0
        for n in range(NT):
            for m in range(n, NT):
                li = A.local_index(m, n)
                if li < 0:
                    continue
                got = store.view(-1, nb, nb)[li].t()
                ref = Lref[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
                if m == n:
                    got, ref = torch.tril(got), torch.tril(ref)
                err = max(err, float((got - ref).abs().max()))
        err /= float(Lref.abs().max())
        if world > 1:
            te = torch.tensor([err], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
            err = float(te.item())
        check = err
        _stage("check done")

    # every rank's one-sided transfers by route (IPC pull over xGMI / host
    # fragments) and payload bytes, gathered for the JSON line; a multi-rank run
    # whose payloads went through host fragments is not the headline path
    comm = []
    if world > 1:
        cs = pa.comm_stats()
        keys = ("get_ipc", "get_fragments", "bytes_pulled_ipc", "bytes_fragments", "gets_queued_max", "gets_inflight_max", "gets_lanes_busy_max")
        rows = gather_rows([int(cs.get(k, 0)) for k in keys])
        comm = [dict(rank=r, **{k: int(v) for k, v in zip(keys, g)}) for r, g in enumerate(rows)]
        # bytes pulled from each peer (rank x source), xGMI link by link
        per_peer = pa.comm_bytes_by_peer() or [0] * world
        peer_rows = gather_rows(per_peer)
        for c, row in zip(comm, peer_rows):
            c["bytes_from_peer"] = row
    devs = pa.devices()
    _stage("fini context")
    ctx.fini()
    _stage("context finalized")
    if world > 1:
        pa.comm_fini()
        _stage("comm finalized")
    out = dict(base)
    out["value"] = round(gflops, 1)
    out["ms_per_step"] = round(ms, 3)
    out["residual"] = float(f"{resid:.3e}")
    out["device_plane"] = planes
    if probe is not None:
        out["ipc_probe"] = probe
    if comm:
        out["comm"] = comm
    est = pa.trsm_estimate_stats(False)
    out["panel_solve"] = {"mode": {0: "inverse", 1: "auto", 2: "blocked"}.get(pa.trsm_inverse_mode(), "?"),
                          "estimates_published": est[0], "decided_on_host": est[1], "device_gate": est[2]}
    if check is not None:
        out["max_rel_error_vs_torch_cholesky"] = check
    gpu_stats = [d for d in devs if d["type"] == pa.DEV_HIP]
    if gpu_stats:
        out["gpu_kernel_launches"] = gpu_stats[0]["kernel_launches"]
        out["gpu_tasks"] = gpu_stats[0]["executed_tasks"]
        if os.environ.get("PARSEC_BENCH_VERBOSE"):
            out["manager_ms"] = {k: round(gpu_stats[0][k], 2) for k in ("ms_complete", "ms_complete_max", "ms_launch")}
    frag = [c["rank"] for c in comm if c["get_fragments"] > 0]
    if frag and not args.allow_host_plane:
        if world > 1:
            dist.destroy_process_group()
        base.update(out)
        fail(4, f"payloads took the host-fragment route on ranks {frag}", {})
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
