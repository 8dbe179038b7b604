"""Ports of the reference's single-process DTD programs (tests/dsl/dtd/*.c),
re-specified over the Python DTD interface: tasks inserting tasks, a task
that yields with HOOK_AGAIN while it inserts (untie), several taskpools waited
separately, taskpools enqueued / dequeued on one context, DONT_TRACK accesses,
NULL tiles, explicit task classes."""
import threading

import pytest


def _ctx(pa, cores=4):
    return pa.init(cores)


def _tiles(pa, n):
    return pa.BlockCyclic(pa.MATRIX_INTEGER, 0, 1, 1, n, 1)


def test_task_inserting_task(pa):
    """dtd_test_task_inserting_task.c: a task body inserts the next tasks of a
    chain into the same taskpool; the chain order is preserved."""
    ctx = _ctx(pa)
    A = _tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    t = tp.tile_of(A, A.data_key([0, 0]))
    seen = []

    def step(task):
        a = task.arg(0)
        seen.append(int(a[0, 0]))
        a[0] += 1
        return 0

    def spawner(task):
        for _ in range(20):
            pa.insert_task(tp, step, [(t, pa.INOUT)])
        return 0

    pa.insert_task(tp, spawner, [(t, pa.INPUT)])
    tp.wait()
    tp.data_flush_all(A)
    ctx.wait()
    assert seen == list(range(20))
    ctx.fini()


def test_untie_task_yields_with_again(pa):
    """dtd_test_untie.c: an inserting task returns HOOK_AGAIN after each batch
    (it is rescheduled and resumes), the inserted tasks run meanwhile."""
    ctx = _ctx(pa)
    A = _tiles(pa, 4)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    tiles = [tp.tile_of(A, A.data_key([i, 0])) for i in range(4)]
    state = {"batch": 0, "calls": 0}
    lock = threading.Lock()
    done = []

    def work(task):
        with lock:
            done.append(task.value_int(0))
        task.arg(1)[0] += 1
        return 0

    def inserter(task):
        state["calls"] += 1
        b = state["batch"]
        if b == 5:
            return pa.HOOK_DONE
        for i in range(4):
            pa.insert_task(tp, work, [(b, pa.VALUE), (tiles[i], pa.INOUT)])
        state["batch"] = b + 1
        return pa.HOOK_AGAIN

    pa.insert_task(tp, inserter, [])
    tp.wait()
    tp.data_flush_all(A)
    ctx.wait()
    assert state["calls"] == 6
    assert sorted(done) == sorted([b for b in range(5) for _ in range(4)])
    for i in range(4):
        assert int(A.tile(i, 0)[0, 0]) == 5
    ctx.fini()


def test_multiple_handle_wait(pa):
    """dtd_test_multiple_handle_wait.c: two DTD taskpools live in one context
    and are waited independently."""
    ctx = _ctx(pa)
    A = _tiles(pa, 2)
    tp1 = pa.dtd_taskpool(ctx)
    tp2 = pa.dtd_taskpool(ctx)
    ctx.start()
    counts = [0, 0]

    def inc(k):
        def body(task):
            task.arg(0)[0] += 1
            counts[k] += 1
            return 0
        body.__name__ = f"inc{k}"
        return body

    t1 = tp1.tile_of(A, A.data_key([0, 0]))
    t2 = tp2.tile_of(A, A.data_key([1, 0]))
    for _ in range(30):
        pa.insert_task(tp1, inc(0), [(t1, pa.INOUT)])
        pa.insert_task(tp2, inc(1), [(t2, pa.INOUT)])
    tp1.data_flush_all(A)
    tp1.wait()
    assert counts[0] == 30
    tp2.data_flush_all(A)
    tp2.wait()
    assert counts[1] == 30
    ctx.wait()
    assert int(A.tile(0, 0)[0, 0]) == 30 and int(A.tile(1, 0)[0, 0]) == 30
    ctx.fini()


def test_tp_enqueue_dequeue(pa):
    """dtd_test_tp_enqueue_dequeue.c: taskpools are added to a running context,
    complete, are removed, and new ones reuse the context."""
    ctx = _ctx(pa)
    A = _tiles(pa, 1)
    ctx.start()
    total = 0
    for rnd in range(4):
        tp = pa.dtd_taskpool(ctx)
        t = tp.tile_of(A, A.data_key([0, 0]))
        for _ in range(10):
            pa.insert_task(tp, lambda task: task.arg(0).__setitem__(0, task.arg(0)[0] + 1) or 0, [(t, pa.INOUT)], name="bump")
        tp.data_flush_all(A)
        tp.wait()
        total += 10
        assert int(A.tile(0, 0)[0, 0]) == total
        tp.close()
    ctx.wait()
    ctx.fini()


def test_flag_dont_track(pa):
    """dtd_test_flag_dont_track.c: accesses flagged DONT_TRACK create no
    dependency, so readers of a tile do not wait for a tracked writer."""
    ctx = _ctx(pa, 4)
    A = _tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    t = tp.tile_of(A, A.data_key([0, 0]))
    gate = threading.Event()
    order = []

    def slow_writer(task):
        gate.wait(10)
        order.append("w")
        return 0

    def untracked_reader(task):
        order.append("r")
        gate.set()
        return 0

    pa.insert_task(tp, slow_writer, [(t, pa.INOUT)])
    pa.insert_task(tp, untracked_reader, [(t, pa.INPUT | pa.DONT_TRACK)])
    tp.wait()
    tp.data_flush_all(A)
    ctx.wait()
    # the untracked reader ran while the writer was still blocked on it
    assert order == ["r", "w"]
    ctx.fini()


def test_null_as_tile(pa):
    """dtd_test_null_as_tile.c: a NULL tile argument yields a None data pointer."""
    ctx = _ctx(pa)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    got = []
    for _ in range(4):
        pa.insert_task(tp, lambda task: got.append(task.arg(0) is None) or 0, [(None, pa.INOUT)], name="null_tile")
    tp.wait()
    ctx.wait()
    assert got == [True] * 4
    ctx.fini()


def test_explicit_task_class(pa):
    """dtd_test_explicit_task_creation.c: a task class created once and
    instances inserted through it (parsec_dtd_create_task_class +
    parsec_dtd_insert_task_with_task_class)."""
    ctx = _ctx(pa)
    A = _tiles(pa, 1)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    tc = tp.task_class("axpy", [(pa.INOUT, pa.PASSED_BY_REF), (pa.VALUE, 4)])
    tp.add_chore(tc, pa.DEV_CPU, lambda task: task.arg(0).__setitem__(0, task.arg(0)[0] + task.value_int(1)) or 0)
    t = tp.tile_of(A, A.data_key([0, 0]))
    for k in range(1, 11):
        tp.insert_task(tc, [(t, pa.INOUT), (k, pa.VALUE)])
    tp.data_flush_all(A)
    tp.wait()
    ctx.wait()
    assert int(A.tile(0, 0)[0, 0]) == 55
    assert tc.name == "axpy" and tc.nb_flows == 1
    ctx.fini()


@pytest.mark.gpu
def test_pushout_flow_returns_home_after_gpu_task(pa):
    """DTD PUSHOUT (reference PARSEC_PUSHOUT): a flow written by a GPU chore is
    copied back to the host when the task completes (device bytes_out grows by
    the tile size before any flush), without the flag it stays on the GPU."""
    ctx = pa.init(2)
    if pa.first_gpu_device_index() < 0:
        pytest.skip("no GPU")
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, 256, 256, 512, 256)
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    gpu = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]
    bytes_tile = 256 * 256 * 8
    t0 = tp.tile_of(A, A.data_key([0, 0]))
    t1 = tp.tile_of(A, A.data_key([1, 0]))
    out0 = gpu["bytes_out"]
    pa.insert_task(tp, None, [(t0, pa.INOUT), (bytes_tile, pa.VALUE, 8), (0, pa.VALUE)], name="memset_plain", gpu="memset")
    tp.wait()
    out1 = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]["bytes_out"]
    pa.insert_task(tp, None, [(t1, pa.INOUT | pa.PUSHOUT), (bytes_tile, pa.VALUE, 8), (0, pa.VALUE)], name="memset_push", gpu="memset")
    tp.wait()
    out2 = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]["bytes_out"]
    tp.data_flush_all(A)
    ctx.wait()
    assert out1 - out0 < bytes_tile
    assert out2 - out1 >= bytes_tile
    assert float(abs(A.tile(1, 0)).max()) == 0.0
    ctx.fini()
