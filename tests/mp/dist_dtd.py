"""Worker: one rank of the distributed DTD collective patterns (every rank
inserts the same task stream, tasks run on the rank of their AFFINITY tile).
argv: rank size job case. Cases mirror the reference's tests/dsl/dtd
broadcast / reduce / allreduce / pingpong / war programs (re-specified).
Tile r (4 doubles) lives on rank r."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import parsec_amd as pa  # noqa: E402


def main():
    rank, size, job, case = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    assert pa.comm_init(rank, size, job, -1) == 0
    ctx = pa.init(2)
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, rank, 4, 1, 4 * size, 1, P=size, Q=1)
    mine = A.tile(rank, 0) if A.rank_of([rank, 0]) == rank else None
    mine[:] = rank + 1
    tp = pa.dtd_taskpool(ctx)
    ctx.start()
    T = [tp.tile_of(A, A.data_key([r, 0])) for r in range(size)]
    expect = None

    def setv(v):
        def body(task):
            task.arg(0)[:] = v
            return 0
        body.__name__ = "setv"
        return body

    def add_into(task):  # arg0 += arg1
        task.arg(0)[:] += task.arg(1)
        return 0

    def copy_from(task):  # arg1 := arg0 (+ arg2 value)
        task.arg(1)[:] = task.arg(0) + task.value_double(2)
        return 0

    def bump(task):  # arg0 += 1 (arg1 only places the task)
        task.arg(0)[:] += 1
        return 0

    if case == "broadcast":
        pa.insert_task(tp, setv(42.0), [(T[0], pa.INOUT | pa.AFFINITY)])
        for r in range(1, size):
            pa.insert_task(tp, copy_from, [(T[0], pa.INPUT), (T[r], pa.INOUT | pa.AFFINITY), (float(r), pa.VALUE)])
        expect = 42.0 + rank
    elif case in ("reduce", "allreduce"):
        for r in range(1, size):
            pa.insert_task(tp, add_into, [(T[0], pa.INOUT | pa.AFFINITY), (T[r], pa.INPUT)])
        total = size * (size + 1) / 2
        if case == "allreduce":
            for r in range(1, size):
                pa.insert_task(tp, copy_from, [(T[0], pa.INPUT), (T[r], pa.INOUT | pa.AFFINITY), (0.0, pa.VALUE)])
            expect = total
        else:
            expect = total if rank == 0 else rank + 1.0
    elif case == "pingpong":
        n = 6 * size
        for k in range(n):
            r = k % size
            if r == 0:
                pa.insert_task(tp, bump, [(T[0], pa.INOUT | pa.AFFINITY)], name="bump0")
            else:
                pa.insert_task(tp, bump, [(T[0], pa.INOUT), (T[r], pa.INPUT | pa.AFFINITY)])
        expect = 1.0 + n if rank == 0 else rank + 1.0
    elif case == "war":
        # every rank snapshots T0, then rank 0 overwrites it: readers see the old value
        for r in range(1, size):
            pa.insert_task(tp, copy_from, [(T[0], pa.INPUT), (T[r], pa.INOUT | pa.AFFINITY), (100.0, pa.VALUE)])
        pa.insert_task(tp, setv(-5.0), [(T[0], pa.INOUT | pa.AFFINITY)])
        expect = -5.0 if rank == 0 else 101.0
    elif case == "multiflow":
        # a remote writer with two written flows (T0 and T1 on rank 1), read on
        # rank 0 right away: both flows of the shadow are activated on rank 0
        # while later insertions race with the arrivals (dtd.cpp)
        def w2(task):
            task.arg(0)[:] += 1
            task.arg(1)[:] += 2
            return 0

        t0, t1 = 1.0, 2.0
        for _ in range(12):
            pa.insert_task(tp, w2, [(T[0], pa.INOUT), (T[1], pa.INOUT | pa.AFFINITY)])
            pa.insert_task(tp, add_into, [(T[0], pa.INOUT | pa.AFFINITY), (T[1], pa.INPUT)])
            t0, t1 = t0 + 1, t1 + 2
            t0 += t1
        expect = t0 if rank == 0 else (t1 if rank == 1 else rank + 1.0)
    elif case == "placement":
        # VALUE | AFFINITY places a task on the rank it names; out-of-range
        # ranks fall back to rank 0 (reference dtd_test_task_placement.c)
        ran = []

        def placed(task):
            ran.append(task.value_int(0))
            return 0

        for r in range(size + 1):
            pa.insert_task(tp, placed, [(r, pa.VALUE | pa.AFFINITY)])
        tp.wait()
        bad = [r for r in ran if (r if r < size else 0) != rank]
        mine[:] = len(ran) if not bad else -1
        expect = 2.0 if rank == 0 else 1.0
    elif case == "null_tile":
        # NULL passed as a tile: the task runs on the inserting rank with a
        # null argument (reference dtd_test_null_as_tile.c)
        ran = []

        def nulltask(task):
            ran.append(task.arg(0) is None)
            return 0

        for _ in range(5):
            pa.insert_task(tp, nulltask, [(None, pa.INOUT)])
        tp.wait()
        mine[:] = sum(ran)
        expect = 5.0
    else:
        raise SystemExit(f"unknown case {case}")
    tp.data_flush_all(A)
    ctx.wait()
    got = float(mine[0, 0])
    ctx.fini()
    pa.comm_fini()
    ok = abs(got - expect) < 1e-12
    print(f"rank {rank} case {case} got {got} expect {expect} {'ok' if ok else 'BAD'}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
