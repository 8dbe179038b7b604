"""Tracing pipeline: task_profiler PINS module -> binary trace per rank ->
parsec_amd.profiling reader / summary / CSV / chrome export, and the DOT
grapher (reference tests/profiling: generate .prof with task_profiler, convert,
validate event counts)."""
import json
import os

import numpy as np
import pytest

from parsec_amd import profiling


def test_trace_roundtrip(pa, tmp_path):
    base = str(tmp_path / "trace")
    pa.mca_set("profile_filename", base)
    pa.mca_set("mca_pins", "task_profiler")
    pa.mca_set("parsec_dot", str(tmp_path / "graph"))
    try:
        ctx = pa.init(3)
    finally:
        pa.mca_unset("profile_filename")
        pa.mca_unset("mca_pins")
        pa.mca_unset("parsec_dot")
    A = pa.BlockCyclic(pa.MATRIX_INTEGER, 0, 1, 1, 4, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()

    def work(task):
        task.arg(0)[0, 0] += 1
        return 0

    for i in range(40):
        t = tp.tile_of(A, A.data_key([i % 4, 0]))
        pa.insert_task(tp, work, [(t, pa.INOUT)], name="traced_work")
    tp.data_flush_all(A)
    ctx.wait()
    ctx.fini()
    path = base + "-0.prof"
    assert os.path.exists(path)
    tr = profiling.read_trace(path)
    assert tr.rank == 0
    summ = profiling.summary([tr])
    assert summ["traced_work"]["count"] == 40
    assert summ["traced_work"]["total_ns"] > 0
    # PINS DATA_FLUSH events (reference parsec_dtd_data_flush.c:391,395): one per flushed tile
    assert summ["DATA_FLUSH"]["count"] == 4
    df = profiling.to_dataframe([tr])
    w = df[df["type"] == "traced_work"]
    assert len(w) == 40 and (w["duration"] >= 0).all()
    assert set(np.unique(w["taskpool_id"])) == {tp.taskpool_id}
    out = tmp_path / "t.json"
    profiling.to_chrome([tr], str(out))
    ev = json.load(open(out))["traceEvents"]
    assert sum(1 for e in ev if e["name"] == "traced_work") == 40
    # DOT grapher: one node per executed task
    dots = [p for p in os.listdir(tmp_path) if p.startswith("graph")]
    assert dots
    profiling.dot_merge([str(tmp_path / d) for d in dots], str(tmp_path / "merged.dot"))
    text = open(tmp_path / "merged.dot").read()
    assert text.startswith("digraph") and text.count("traced_work") >= 40


def test_trace_streaming_writer(pa, tmp_path):
    """profile_buffer_events=16: every stream's buffer is handed to the writer
    thread many times during the run (bounded memory, reference profiling.c
    helper-thread flush); the assembled trace still holds every event, the spill
    files are gone, and the header carries the process rusage."""
    base = str(tmp_path / "spill")
    pa.mca_set("profile_filename", base)
    pa.mca_set("profile_buffer_events", "16")
    pa.mca_set("mca_pins", "task_profiler")
    try:
        ctx = pa.init(2)
    finally:
        for k in ("profile_filename", "profile_buffer_events", "mca_pins"):
            pa.mca_unset(k)
    A = pa.BlockCyclic(pa.MATRIX_INTEGER, 0, 1, 1, 8, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    for i in range(300):
        pa.insert_task(tp, lambda task: 0, [(tp.tile_of(A, A.data_key([i % 8, 0])), pa.INOUT)], name="spilled_work")
    tp.data_flush_all(A)
    ctx.wait()
    ctx.fini()
    tr = profiling.read_trace(base + "-0.prof")
    assert profiling.summary([tr])["spilled_work"]["count"] == 300
    assert not [p for p in os.listdir(tmp_path) if p.endswith(".tmp")]
    infos = dict(tr.infos)
    assert float(infos["ru_utime_s"]) >= 0 and float(infos["ru_maxrss_kb"]) > 0


def test_comm_trace_payload_sizes(pa, tmp_path):
    """Distributed run with a trace per rank: every payload has a COMM_DATA_SND
    span at its sender and a COMM_DATA_RCV span at its receiver with the same
    byte count (the check of the reference's tests/profiling/check-comms.py)."""
    import subprocess
    import sys
    import uuid

    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp", "dist_dpotrf.py")
    base = str(tmp_path / "comm")
    job = "pc" + uuid.uuid4().hex[:10]
    env = dict(os.environ, PARSEC_MCA_device_hip_enabled="0", PARSEC_MCA_profile_filename=base, PARSEC_MCA_mca_pins="task_profiler")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", job, "256", "32", "2", "1"], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, env=env) for r in range(2)]
    for p in procs:
        out, _ = p.communicate(timeout=120)
        assert p.returncode == 0, out
    traces = [profiling.read_trace(f"{base}-{r}.prof") for r in range(2)]
    rows = profiling.intervals(traces)
    snd = [(r["rank"], r["peer"], r["bytes"]) for r in rows if r["type"] == "COMM_DATA_SND"]
    rcv = [(r["peer"], r["rank"], r["bytes"]) for r in rows if r["type"] == "COMM_DATA_RCV"]
    assert snd and sorted(snd) == sorted(rcv)
    assert all(b == 32 * 32 * 8 for *_, b in snd)
    assert any(r["type"] == "COMM_ACTIVATE" for r in rows)
    # PINS ACTIVATE_CB spans (reference remote_dep_mpi.c:1838,1887): every
    # received activation runs its callback inside one
    assert any(r["type"] == "ACTIVATE_CB" for r in rows)


def test_dagtools_on_recorded_cholesky_dag(pa, tmp_path):
    """DAG tools (reference tools/dagenum.c, grapher.c): the DOT written by the
    grapher for a tiled Cholesky has every task, is acyclic, and its critical
    path is POTRF -> TRSM -> SYRK per panel (3 NT - 2 tasks)."""
    from parsec_amd import dagtools

    NT, nb = 5, 4
    pa.mca_set("parsec_dot", str(tmp_path / "chol"))
    pa.mca_set("device_hip_enabled", "0")
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("parsec_dot")
        pa.mca_unset("device_hip_enabled")
    N = NT * nb
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
    S = np.random.default_rng(3).standard_normal((N, N))
    S = S @ S.T + N * np.eye(N)
    for m in range(NT):
        for n in range(NT):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
            A.mark_host_modified(m, n)
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    ctx.fini()
    dots = [str(tmp_path / p) for p in os.listdir(tmp_path) if p.startswith("chol")]
    g = dagtools.read_dot(dots)
    st = g.stats()
    assert st["nodes"] == NT * (NT + 1) * (NT + 2) // 6
    assert st["acyclic"] and st["roots"] == 1
    assert st["critical_path"] == 3 * NT - 2
    assert dagtools.main(["stats"] + dots) == 0
    classes = {g.class_of(x) for x in g.nodes}
    assert len(classes) >= 3


def test_live_properties_publisher(pa, tmp_path):
    """Live properties (reference tools/aggregator_visu over the shm dictionary):
    with profile_properties_shm the runtime refreshes the segment while it runs;
    parsec_amd.aggregator reads the device counters and user properties."""
    import uuid

    from parsec_amd import aggregator

    name = "pamd_props_" + uuid.uuid4().hex[:8]
    pa.mca_set("profile_properties_shm", name)
    pa.mca_set("profile_properties_period_ms", "10")
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("profile_properties_shm")
        pa.mca_unset("profile_properties_period_ms")
    try:
        pa.properties_set("app.iteration", 7.0)
        A = pa.BlockCyclic(pa.MATRIX_INTEGER, 0, 1, 1, 4, 1)
        tp = pa.dtd_taskpool(ctx)
        ctx.start()
        for i in range(64):
            pa.insert_task(tp, lambda task: 0, [(tp.tile_of(A, A.data_key([i % 4, 0])), pa.INOUT)], name="props_work")
        tp.data_flush_all(A)
        ctx.wait()
        import time

        time.sleep(0.05)
        seq, vals = aggregator.read(name)
        assert seq >= 1
        assert vals.get("app.iteration") == 7.0
        assert any(k.startswith("device.") and k.endswith(".executed_tasks") for k in vals)
        assert "runtime.threads" in vals
        ctx.fini()
        seq2, vals2 = aggregator.read(name)  # final snapshot written at fini
        cpu = [v for k, v in vals2.items() if k.endswith(".executed_tasks")]
        assert max(cpu) >= 64
        assert aggregator.main([name, "--count", "1", "--interval", "0"]) == 0
    finally:
        try:
            os.unlink(os.path.join("/dev/shm", name))
        except OSError:
            pass


def test_standalone_profiling_c_threads(pa, tmp_path):
    """Standalone profiling API from C without a runtime context (port of the
    reference's tests/profiling-standalone/sp-demo.c and sp-perf.c): 4 threads,
    one stream each (parsec_profiling_stream_init), per-stream and global
    key / values, 10 begin / end pairs per thread, the B events' info structure
    {int i; double d} decoded from the trace; the perf mode traces 2 x 20000
    events per thread."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "sp_demo")
    cmd = ["gcc", "-std=gnu99", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{root}/include", os.path.join(root, "tests", "capi", "sp_demo.c"), "-o", exe,
           "-lpthread", f"-L{root}/parsec_amd/lib", "-lparsec_amd", f"-Wl,-rpath,{root}/parsec_amd/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe, "demo", str(tmp_path / "sp")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "sp-demo done" in r.stdout, r.stdout + r.stderr
    tr = profiling.read_trace(str(tmp_path / "sp-0.prof"))
    assert tr.infos["This is a global information key"] == "This is the global information value"
    assert tr.infos["hr_id"] == "Demonstration of basic PaRSEC profiling system"
    names = sorted(s["name"] for s in tr.streams)
    assert names == [f"This is the name of thread {i}" for i in range(4)]
    assert all(s["infos"] == {"This is a thread-specific information key": "This is the corresponding value"} for s in tr.streams)
    rows = profiling.intervals([tr])
    assert len(rows) == 40 and {r["type"] for r in rows} <= {"Event A", "Event B"}
    for r in rows:
        assert r["end"] >= r["begin"]
        if r["type"] == "Event B":
            assert r["i"] == r["event_id"] and r["d"] == float(r["stream"].split()[-1])
    r = subprocess.run([exe, "perf", str(tmp_path / "spp"), "20000"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ns per event" in r.stdout, r.stdout + r.stderr
    print(r.stdout.strip().splitlines()[0])
    tr = profiling.read_trace(str(tmp_path / "spp-0.prof"))
    assert sum(len(s["events"]) for s in tr.streams) == 4 * 2 * 20000


def _check_async(traces, nb):
    """tests/profiling/check-async.py of the reference, over parsec_amd.profiling
    intervals instead of its HDF5 tables: one STARTUP, one FULL_RESCHED, NB
    FULL_ASYNC, 2*NB ASYNC (each body runs twice), RESCHED executions mutually
    exclusive and inside FULL_RESCHED (except the first one's begin and the
    last one's end), ASYNC(k)'s first run ending and second run beginning inside
    FULL_ASYNC(k)."""
    import pandas as pd

    ev = pd.DataFrame(profiling.intervals(traces))
    assert int(traces[0].infos["NB"]) == nb
    cnt = ev.type.value_counts()
    assert cnt.get("STARTUP", 0) == 1 and cnt.get("FULL_RESCHED", 0) == 1, cnt
    assert cnt.get("FULL_ASYNC", 0) == nb and cnt.get("ASYNC", 0) == 2 * nb, cnt
    full = ev[ev.type == "FULL_RESCHED"].iloc[0]
    res = ev[ev.type == "RESCHED"].sort_values("begin")
    assert len(res) >= 1
    before = res[res.begin < full.begin]
    after = res[res.end > full.end]
    assert len(before) <= 1 and len(after) <= 1, (before, after)
    for _, e in before.iterrows():
        assert full.begin <= e.end <= full.end
    for _, e in after.iterrows():
        assert full.begin <= e.begin <= full.end
    b, e = res.begin.to_numpy(), res.end.to_numpy()
    assert (b[1:] > e[:-1]).all(), "two RESCHED executions overlap"
    fa = ev[ev.type == "FULL_ASYNC"].set_index("event_id")
    asy = ev[ev.type == "ASYNC"].sort_values("begin")
    for k, g in asy.groupby("k"):
        assert len(g) == 2, (k, g)
        ref = fa.loc[k]
        first, second = g.iloc[0], g.iloc[1]
        assert ref.begin <= first.end <= ref.end, k
        assert ref.begin <= second.begin <= ref.end, k
    assert sorted(asy.k.unique()) == list(range(nb))


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
@pytest.mark.parametrize("nb,cores", [(100, 4), (1000, 8), (300, 1)])
def test_reference_async_profile(pa, tmp_path, nb, cores):
    """The reference's tests/profiling/async.jdf, unmodified: bodies that return
    PARSEC_HOOK_RETURN_ASYNC and are put back by another task's
    __parsec_schedule, a body that returns AGAIN until they all ran once, user
    streams per thread (parsec_profiling_stream_init) with begin / end events
    that cross threads, profiling_save_iinfo, and the task_profiler's per-local
    columns; traced with --mca profile_filename / mca_pins task_profiler, as
    Testings.cmake:20 runs it, and checked as check-async.py does."""
    import subprocess

    from parsec_amd import ptgpp

    exe = ptgpp.build_program(os.path.join(REF, "tests/profiling/async.jdf"), str(tmp_path), cxxflags=ptgpp.C_BODIES + (f"-I{REF}",))
    r = subprocess.run([exe, str(nb), "--", "--mca", "profile_filename", str(tmp_path / "async"), "--mca", "mca_pins", "task_profiler",
                        "--mca", "runtime_num_cores", str(cores)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PARSEC_MCA_device_hip_enabled="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    _check_async([profiling.read_trace(str(tmp_path / "async-0.prof"))], nb)
