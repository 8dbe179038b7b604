"""Multi-process (one process per rank) runs of the distributed engine on CPU:
shared-memory active messages, host-data fragments, broadcast trees,
local / four-counter termination (reference tests: collections/*:mp, dsl/ptg :mp)."""
import os
import subprocess
import sys
import uuid

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "mp", "dist_dpotrf.py")


def run_ranks(nranks, *args, timeout=120, worker=WORKER, env_extra=None):
    job = "pt" + uuid.uuid4().hex[:10]
    env = dict(os.environ, PARSEC_MCA_device_hip_enabled="0", **(env_extra or {}))
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(nranks), job, *map(str, args)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
             for r in range(nranks)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.mark.parametrize("nranks,P,Q,topo,termdet", [
    (2, 2, 1, "star", "local"),
    (2, 1, 2, "star", "fourcounter"),
    (4, 2, 2, "chain", "local"),
    (4, 2, 2, "binomial", "fourcounter"),
    (8, 4, 2, "binomial", "fourcounter"),  # the process grid bench.py uses on 8 GPUs
])
def test_distributed_dpotrf(pa, nranks, P, Q, topo, termdet):
    outs = run_ranks(nranks, 512, 64, P, Q, "lfq", topo, termdet)
    for rc, out in outs:
        assert rc == 0, out


@pytest.mark.parametrize("nranks,P,Q,mode", [
    (2, 2, 1, {}),
    (4, 2, 2, {"PARSEC_MCA_ptg_deps_mask": "1"}),
    (3, 3, 1, {"PARSEC_MCA_ptg_dep_management": "dynamic-hash-table"}),
    (4, 2, 2, {"PARSEC_DPOTRF_FUSE_SYRK": "1"}),  # SYRK(k-1,k) inside POTRF(k): TRSM(k,k-1) -> POTRF(k) crosses ranks
])
def test_distributed_dpotrf_jdf(pa, nranks, P, Q, mode):
    """The ptgpp-compiled dpotrf_L.jdf over several ranks (remote activations
    into index-array / hash storage, counter / mask tracking)."""
    outs = run_ranks(nranks, 384, 64, P, Q, "lfq", "star", "local", env_extra=dict(mode, DPOTRF_TASKPOOL="jdf"))
    for rc, out in outs:
        assert rc == 0, out


@pytest.mark.parametrize("nranks,pad", [(2, 0), (3, 1)])
def test_distributed_diag_band_to_rect(pa, nranks, pad):
    """diag_band_to_rect.jdf with the band on a P x 1 grid and the target row on
    a 1 x Q grid: the source tiles travel to the target tiles' owners."""
    outs = run_ranks(nranks, 6, 5, pad, worker=os.path.join(HERE, "mp", "dist_band.py"))
    for rc, out in outs:
        assert rc == 0 and "band ok" in out, out


@pytest.mark.parametrize("aggregate", ["1", "0"])
def test_distributed_backpressure_aggregation(pa, aggregate):
    """Tiny shared-memory rings and a slow receiver (comm_shm_debug_delay_us)
    force activations into the per-peer priority backlog; with runtime_comm_aggregate they leave packed in one message
    (reference remote_dep_mpi.c:1089-1139, runtime_comm_aggregate). The
    factorization stays exact either way."""
    outs = run_ranks(4, 256, 8, 2, 2, "lfq", "star", "local",
                     env_extra={"PARSEC_MCA_comm_shm_ring_bytes": "8192", "PARSEC_MCA_runtime_comm_aggregate": aggregate,
                                "PARSEC_MCA_comm_shm_debug_delay_us": "300",
                                "DIST_PRINT_COMM_STATS": "1"})
    stats = []
    for rc, out in outs:
        assert rc == 0, out
        line = [x for x in out.splitlines() if x.startswith("comm_stats")][0]
        stats.append(dict(kv.split("=") for kv in line.split()[1:]))
    assert sum(int(s["backlogged"]) for s in stats) > 0
    if aggregate == "1":
        assert sum(int(s["aggregates"]) for s in stats) > 0
        assert all(int(s["aggregated_msgs"]) >= 2 * int(s["aggregates"]) for s in stats)
    else:
        assert sum(int(s["aggregates"]) for s in stats) == 0


@pytest.mark.parametrize("sched", ["gd", "ll", "ap"])
def test_distributed_other_schedulers(pa, sched):
    outs = run_ranks(2, 384, 64, 2, 1, sched, "star", "local")
    for rc, out in outs:
        assert rc == 0, out


@pytest.mark.parametrize("case", ["broadcast", "reduce", "allreduce", "pingpong", "war", "multiflow", "placement", "null_tile"])
@pytest.mark.parametrize("nranks", [2, 3])
def test_distributed_dtd_patterns(pa, case, nranks):
    """Distributed DTD: one writer read on every rank, reduction into rank 0,
    all-reduce, a tile bouncing between ranks, readers-before-writer across
    ranks (reference tests/dsl/dtd broadcast / reduce / allreduce / pingpong / war)."""
    outs = run_ranks(nranks, case, worker=os.path.join(HERE, "mp", "dist_dtd.py"))
    for rc, out in outs:
        assert rc == 0, out


def test_launcher_kills_survivors_on_failure():
    """mpiexec semantics: one rank failing ends the whole job."""
    import time

    from parsec_amd import launch

    prog = "import os, sys, time; r = int(os.environ['PARSEC_COMM_RANK']); sys.exit(3) if r == 1 else time.sleep(60)"
    t0 = time.monotonic()
    rc = launch.launch(3, [sys.executable, "-c", prog], timeout=50)
    assert rc == 3
    assert time.monotonic() - t0 < 20


@pytest.mark.parametrize("taskpool", ["jdf", "ir"])
@pytest.mark.parametrize("nranks,P,Q,M,N", [(2, 2, 1, 96, 96), (3, 3, 1, 112, 80), (4, 2, 2, 96, 128)])
def test_distributed_dgeqrf(pa, tmp_path, nranks, P, Q, M, N, taskpool):
    """QR over P x Q ranks (the ptgpp-compiled dgeqrf.jdf and the hand-built IR):
    the TS chains write R(k,k) / A(k,n) from remote ranks, so the final versions
    must travel back to the owning rank."""
    import numpy as np

    outs = run_ranks(nranks, M, N, 16, P, Q, str(tmp_path), worker=os.path.join(HERE, "mp", "dist_qr.py"), env_extra={"QR_TASKPOOL": taskpool})
    for rc, out in outs:
        assert rc == 0, out
    R = sum(np.load(tmp_path / f"R{r}.npy") for r in range(nranks))
    S = np.random.default_rng(5).standard_normal((M, N))
    G = S.T @ S
    assert np.linalg.norm(R.T @ R - G) / np.linalg.norm(G) < 1e-13


@pytest.mark.parametrize("nranks,P,Q,M,N,dom", [(2, 2, 1, 128, 96, 2), (4, 2, 2, 160, 128, 2), (4, 4, 1, 192, 96, 1), (3, 3, 1, 112, 80, 3)])
def test_distributed_dgeqrf_hqr(pa, tmp_path, nranks, P, Q, M, N, dom):
    """Hierarchical QR over P x Q ranks: TS domains and TT trees inside a process
    row, TT binary tree across the P process rows (the only cross-rank kills)."""
    import numpy as np

    outs = run_ranks(nranks, M, N, 16, P, Q, str(tmp_path), dom, worker=os.path.join(HERE, "mp", "dist_qr.py"))
    for rc, out in outs:
        assert rc == 0, out
    R = sum(np.load(tmp_path / f"R{r}.npy") for r in range(nranks))
    S = np.random.default_rng(5).standard_normal((M, N))
    G = S.T @ S
    assert np.linalg.norm(R.T @ R - G) / np.linalg.norm(G) < 1e-13


@pytest.mark.parametrize("nranks,method,shape", [
    (2, "ptg", "8 8 5 7 17 13 3 5 9 2"),          # general: different tile sizes, unaligned window
    (4, "ptg", "7 9 11 6 50 41 2 11 13 20"),
    (4, "ptg", "8 8 8 8 40 32 8 16 24 0"),        # tile aligned, same tiles: the reshuffle taskpool
    (3, "ptg", "6 10 10 6 60 50 4 6 1 9"),
    (4, "dtd", "7 9 11 6 50 41 2 11 13 20"),
])
def test_distributed_redistribute(pa, nranks, method, shape):
    """PTG redistribute.jdf / redistribute_reshuffle.jdf between two different
    process grids (reference tests/collections/redistribute), and the DTD form."""
    outs = run_ranks(nranks, method, *shape.split(), worker=os.path.join(HERE, "mp", "dist_redistribute.py"))
    for rc, out in outs:
        assert rc == 0 and "bad 0" in out, out
    assert sum(int(out.split("checked ")[1].split()[0]) for _, out in outs) == int(shape.split()[4]) * int(shape.split()[5])


def _bench_ranks(nranks, extra, timeout=240):
    """bench.py --device cpu as `nranks` processes (the env torchrun would give
    them): returns [(returncode, stdout, stderr)] in rank order."""
    import random

    port = str(29700 + random.randint(0, 250))
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   PARSEC_MCA_device_hip_enabled="0", TORCHELASTIC_RUN_ID="t" + uuid.uuid4().hex[:6] if r == 0 else "")
        procs.append(env)
    rid = procs[0]["TORCHELASTIC_RUN_ID"]
    run = []
    for env in procs:
        env["TORCHELASTIC_RUN_ID"] = rid
        run.append(subprocess.Popen([sys.executable, bench, "--gpus", str(nranks), "--size", "768", "--nb", "128", "--steps", "1",
                                     "--warmup", "0", "--device", "cpu", "--cores", "2", *extra],
                                    stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    try:
        for p in run:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    finally:
        for p in run:
            if p.poll() is None:
                p.kill()
    return outs


def test_bench_json_before_failing_exit(pa):
    """bench.py on a multi-rank job whose device plane is not IPC (here: CPU
    ranks, every peer unprobed) prints its JSON line -- device plane and the
    rank x peer probe table -- BEFORE exiting 3, so a failed 8-GPU run still
    reports which pair failed; with --allow-host-plane the same job runs, and
    the line carries the per-peer payload bytes."""
    import json

    outs = _bench_ranks(2, [])
    assert [rc for rc, _, _ in outs] == [3, 3], [(rc, e[-800:]) for rc, _, e in outs]
    line = [l for l in outs[0][1].splitlines() if l.startswith("{")]
    assert line, outs[0]
    out = json.loads(line[-1])
    assert out["value"] is None and "device plane is not ipc" in out["error"]
    assert [p["plane"] for p in out["device_plane"]] == ["host", "host"]
    assert out["ipc_probe"]["codes"] == [[0, -1], [-1, 0]]
    outs = _bench_ranks(2, ["--allow-host-plane"])
    assert [rc for rc, _, _ in outs] == [0, 0], [(rc, e[-800:]) for rc, _, e in outs]
    out = json.loads([l for l in outs[0][1].splitlines() if l.startswith("{")][-1])
    assert out["value"] > 0 and out["residual"] < 1e-12
    for r, c in enumerate(out["comm"]):
        assert c["get_fragments"] > 0 and sum(c["bytes_from_peer"]) == c["bytes_fragments"], c
        assert c["bytes_from_peer"][r] == 0
