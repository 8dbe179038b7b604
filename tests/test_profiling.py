"""Tracing pipeline: task_profiler PINS module -> binary trace per rank ->
parsec_amd.profiling reader / summary / CSV / chrome export, and the DOT
grapher (reference tests/profiling: generate .prof with task_profiler, convert,
validate event counts)."""
import json
import os

import numpy as np

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
