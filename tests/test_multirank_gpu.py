"""Multi-rank runs of the distributed device data plane on one MI355X: 2, 4 and
8 processes (one per "GPU" of a P x Q grid) all drive GPU 0, and every remote
tile moves HBM -> HBM through the communication engine's one-sided get (the
engine maps the sender's allocation through HIP IPC and pulls it; the get's
PUT_END notification releases the source).
Reference: collections/*:mp and dsl/* :mp tests run with mpiexec -n 2|4|8
(tests/collections/Testings.cmake:5-6, remote_dep.c:454-591).

Oracle note: every rank checks its tiles against a HOST (LAPACK) Cholesky.
torch.linalg.cholesky on the GPU returns wrong factors now and then when several
processes share one MI355X, also with this runtime never imported
(profiles/r3_oracle_root_cause.txt, scripts/oracle_probe.py); the runtime's own
factor matched the host reference to 1e-15 every time."""
import os
import subprocess
import sys
import tempfile
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "mp", "gpu_dist.py")


def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(case, nranks, *args, timeout=100, env_extra=None):
    job = "g" + uuid.uuid4().hex[:10]
    env = dict(os.environ, PYTHONUNBUFFERED="1", **(env_extra or {}))
    procs = [subprocess.Popen([sys.executable, WORKER, case, str(r), str(nranks), job, *map(str, args)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, start_new_session=True)
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
                p.wait()
    for rc, out in outs:
        print(out.strip().splitlines()[-1] if out.strip() else "")
    return outs


# The IPC pull routes. "gather" (the default, comm_ipc_copy_mode 3, the route
# of peers on distinct GPUs too): the pulls of a progress pass leave in ONE
# multi-source gather kernel, one transfer per source peer; on this 1-GPU box
# every peer shares the GPU and the gathers alternate over 2 streams.
# "copy-engine": hipMemcpyAsync per pull on the GPU's one shared copy stream
# (the fall-back of a peer whose probe kernel read failed).
ROUTES = {
    "gather": {},
    "copy-engine": {"PARSEC_MCA_comm_ipc_copy_mode": "0", "PARSEC_MCA_comm_ipc_streams": "1"},
}


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("nranks,P,Q", [(2, 2, 1), (4, 2, 2), (8, 4, 2)])
def test_dpotrf_multirank_ipc(pa, nranks, P, Q, route):
    """N=8192, nb=512 Cholesky over P x Q ranks (the 8-rank grid is the one
    bench.py uses on 8 GPUs), every rank checking its tiles of L, through both
    IPC pull routes."""
    _gpu()
    outs = _run("dpotrf", nranks, 8192, 512, P, Q, env_extra={"EXPECT_PLANE": "ipc", **ROUTES[route]})
    # every rank's warnings in the message: the rank whose IPC start-up failed
    # names its own error code
    notes = "\n".join(f"[{r}] {l}" for r, (_, o) in enumerate(outs) for l in o.splitlines() if "warning" in l or "error" in l.lower() or "status" in l)
    for rc, out in outs:
        assert rc == 0, out + "\n" + notes
    # the remote tiles really moved GPU to GPU through the engine's IPC route,
    # none through host fragments
    last = [o.strip().splitlines()[-1] for _, o in outs]
    gets = [int(l.split(" gets ipc ")[-1].split()[0]) for l in last]
    frags = [int(l.split(" fragments ")[-1].split()[0]) for l in last]
    assert sum(gets) > 0 and sum(frags) == 0, last


def test_dpotrf_host_plane_request(pa):
    """comm_device_plane=host: every rank stages device tiles through host
    fragments (the route a failed IPC start-up falls back to) and the factor is
    still right; no payload takes the IPC route."""
    _gpu()
    outs = _run("dpotrf", 2, 2048, 256, 2, 1, env_extra={"PARSEC_MCA_comm_device_plane": "host", "EXPECT_PLANE": "host"})
    for rc, out in outs:
        assert rc == 0, out
    last = [o.strip().splitlines()[-1] for _, o in outs]
    assert all(" gets ipc 0 " in l for l in last), last
    assert sum(int(l.split(" fragments ")[-1].split()[0]) for l in last) > 0, last


def test_dgeqrf_two_ranks_ipc(pa):
    """1D row-cyclic QR over 2 ranks: R assembled from both ranks satisfies R^T R = A^T A
    (the R(k,k) of each TS chain is written back from the remote rank)."""
    _gpu()
    import torch

    N, nb = 2048, 256
    with tempfile.TemporaryDirectory() as d:
        for rc, out in _run("dgeqrf", 2, N, nb, 2, d):
            assert rc == 0, out
        R = sum(np.load(os.path.join(d, f"R{r}.npy")) for r in range(2))
    g = torch.Generator().manual_seed(77)
    A = (torch.rand((N, N), dtype=torch.float64, generator=g) - 0.5).numpy()
    AtA = A.T @ A
    assert np.linalg.norm(R.T @ R - AtA) / np.linalg.norm(AtA) < 1e-12


def test_dgeqrf_hqr_2x2_ipc(pa):
    """Hierarchical QR on a 2 x 2 process grid (4 ranks sharing the GPU): TS
    domains and TT merges inside each process row on the GPU kernels, the TT
    kill across the two process rows through the device plane; R^T R = A^T A."""
    _gpu()
    import torch

    N, nb = 2048, 256
    with tempfile.TemporaryDirectory() as d:
        for rc, out in _run("dgeqrf", 4, N, nb, 2, d, 2, 2):
            assert rc == 0, out
        R = sum(np.load(os.path.join(d, f"R{r}.npy")) for r in range(4))
    g = torch.Generator().manual_seed(77)
    A = (torch.rand((N, N), dtype=torch.float64, generator=g) - 0.5).numpy()
    AtA = A.T @ A
    assert np.linalg.norm(R.T @ R - AtA) / np.linalg.norm(AtA) < 1e-12


@pytest.mark.parametrize("route", list(ROUTES))
def test_stencil_four_ranks_ipc(pa, route):
    """DTD 3D stencil over 4 ranks with GPU bodies: halo faces cross ranks
    through the device plane and STAY on the device: the receiving rank's
    shadow version is a device copy (csrc/dtd/dtd.cpp shadow_copy_new), so the
    runtime copies zero bytes device -> host and writes nothing back to host
    during the sweeps, while faces did arrive through IPC gets."""
    _gpu()
    for rc, out in _run("stencil", 4, 48, 40, 36, 16, 6, env_extra=ROUTES[route]):
        assert rc == 0, out
        line = next(l for l in out.splitlines() if " halo d2h " in l)
        f = line.split()
        v = {f[i]: int(f[i + 1]) for i in range(3, len(f) - 1, 2)}
        assert v["d2h"] == 0 and v["writeback"] == 0, line
        assert v["get_ipc"] > 0, line
        print(line)


@pytest.mark.parametrize("route", list(ROUTES))
def test_comm_engine_c_program_gpu_memory(tmp_path, pa, route):
    """CE get / put between GPU buffers of two processes (both on GPU 0): the
    registrations export the allocations through HIP IPC and every transfer is
    one device copy on the copy stream (ports dtd_test_ce.c to device memory)."""
    import subprocess

    from parsec_amd import launch

    _gpu()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "ce_capi_gpu")
    cmd = ["gcc", "-std=c99", "-O1", "-DCE_WITH_HIP", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{root}/include",
           os.path.join(root, "tests", "capi", "ce_capi.c"), "-o", exe, f"-L{root}/parsec_amd/lib", "-lparsec_amd",
           f"-Wl,-rpath,{root}/parsec_amd/lib", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rc, outs = launch.launch(2, [exe, "gpu"], timeout=120, capture=True, env={"PARSEC_COMM_GPU": "0", **ROUTES[route]})
    assert rc == 0, outs
    text = "".join(o for o, _ in outs)
    assert text.count("ce ok") == 2 and "[1] GET ok" in text and "[1] PUT ok" in text, text
    assert "[1] MIXED GET ok" in text and "[1] MIXED PUT ok" in text, text


@pytest.mark.parametrize("route", list(ROUTES))
def test_headline_tile_size_8_ranks_shared_gpu(pa, route):
    """The headline tile size (nb=1024) on the 8-rank P4xQ2 grid bench.py uses on
    8 GPUs, N=16384, all ranks on the box's one GPU: bench.py's distributed
    backward-error probe (every rank's tiles, two all-reduces) must pass, and
    its JSON line carries every rank's transfers by route (bench.py exits
    non-zero if any payload took the host-fragment route)."""
    _gpu()
    import json

    port = 29600 + (os.getpid() + (7 if route != "gather" else 0)) % 300
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "8", "--size", "16384", "--nb", "1024",
           "--steps", "1", "--warmup", "0", "--share-gpu", "--cores", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, start_new_session=True, env=dict(os.environ, **ROUTES[route]))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    print(line[:200])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"].startswith("2D block-cyclic P4xQ2")
    assert out["residual"] < 1e-12
    comm = out["comm"]
    assert len(comm) == 8 and all(c["get_fragments"] == 0 for c in comm), comm
    assert sum(c["get_ipc"] for c in comm) > 0 and sum(c["bytes_pulled_ipc"] for c in comm) > 0, comm
    # every pair passed every probe route; bytes by source peer add up
    assert out["ipc_probe"]["codes"] == [[0] * 8 for _ in range(8)], out["ipc_probe"]
    for r, c in enumerate(comm):
        assert sum(c["bytes_from_peer"]) == c["bytes_pulled_ipc"] and c["bytes_from_peer"][r] == 0, c
    # pulls from distinct source ranks were in flight together (lanes)
    assert max(c["gets_lanes_busy_max"] for c in comm) >= 2, comm
    # exactly one pull per (tile, receiving rank): the POTRF(k) panel is ONE
    # packed tile (W with L(k,k)^T above the diagonal), so the panel volume is
    # 42 tiles here where the round-5 DAG (W and L(k,k) apart) pulled 84
    w_tiles, c_tiles = _dpotrf_remote_tiles(16, lambda m, n: (m % 4) * 2 + (n % 2))
    assert (w_tiles, c_tiles) == (42, 394)
    assert sum(c["bytes_pulled_ipc"] for c in comm) == (w_tiles + c_tiles) * 1024 * 1024 * 8, comm


def _dpotrf_remote_tiles(NT, owner):
    """Remote tile transfers of dpotrf_L.jdf (FUSE 0) under the owner map: the
    panel tile of POTRF(k) to every other rank owning a TRSM(m, k), and each
    TRSM(m, k) output to every other rank owning one of its SYRK / GEMM
    consumers; a rank receives a datum once whatever the number of its readers."""
    w = c = 0
    for k in range(NT):
        w += len({owner(m, k) for m in range(k + 1, NT)} - {owner(k, k)})
        for m in range(k + 1, NT):
            readers = {owner(m, m)} | {owner(m, n) for n in range(k + 1, m)} | {owner(r, m) for r in range(m + 1, NT)}
            c += len(readers - {owner(m, k)})
    return w, c


def test_bench_probe_failure_reported(pa):
    """comm_ipc_probe_fail=2:1: rank 2's open of rank 1's probe buffer fails,
    so every rank falls back to the host plane; bench.py prints its JSON line
    (device plane per rank, the rank x peer probe table with the failed pair)
    before exiting non-zero."""
    _gpu()
    import json

    port = 29600 + (os.getpid() + 13) % 300
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "4", "--size", "4096", "--nb", "512",
           "--steps", "1", "--warmup", "0", "--share-gpu", "--cores", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, start_new_session=True,
                       env=dict(os.environ, PARSEC_MCA_comm_ipc_probe_fail="2:1"))
    assert r.returncode != 0, r.stdout[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out["value"] is None and "not ipc" in out["error"], out
    codes = out["ipc_probe"]["codes"]
    assert codes[2][1] == 1, codes  # open failed
    assert all(codes[a][b] == 0 for a in range(4) for b in range(4) if (a, b) != (2, 1)), codes
    assert all(p["plane"] == "host" for p in out["device_plane"]), out["device_plane"]
