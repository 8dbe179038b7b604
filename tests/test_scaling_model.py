"""The DPOTRF scaling model (scripts/scaling_model.py) behind
profiles/r4_scaling_prediction.txt: the graph drains, one rank moves no bytes,
and more ranks never predict less than the critical-path bound allows."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("scaling_model", os.path.join(ROOT, "scripts", "scaling_model.py"))
sm = importlib.util.module_from_spec(spec)
spec.loader.exec_module(sm)


def test_grid_matches_bench():
    assert [sm.grid_of(n) for n in (1, 2, 4, 8)] == [(1, 1), (2, 1), (2, 2), (4, 2)]


def test_one_rank_is_work_bound():
    NT, nb = 12, 1024
    out = sm.simulate(NT, nb, 1, 1, gemm_tf=66.0, potrf_us=0.0, link_gbs=50.0, lat_us=25.0)
    assert out["xgmi_GB"] == 0
    # with a free critical lane the bulk server never idles once started
    g = 2.0 * nb ** 3 / 66e12 * 1e6
    work = sum((NT - k - 1) * (g + g / 2 / 0.85) + (NT - k - 1) * (NT - k - 2) / 2 * g for k in range(NT))
    assert abs(out["span_ms"] * 1e3 - work) / work < 0.02


def test_more_ranks_more_throughput_and_traffic():
    NT, nb = 16, 1024
    prev = None
    for r in (1, 2, 4, 8):
        P, Q = sm.grid_of(r)
        out = sm.simulate(NT, nb, P, Q, gemm_tf=66.0, potrf_us=350.0, link_gbs=50.0, lat_us=25.0)
        chain = sm.critical_path_us(NT, 350.0, 2.0 * nb ** 3 / 66e12 * 1e6, nb ** 3 / 66e12 * 1e6 / 0.85, nb * nb * 8 / 50e9 * 1e6 + 25.0, P, Q)
        assert out["span_ms"] * 1e3 >= chain * 0.999
        if prev:
            assert out["tflops"] >= prev["tflops"] * 0.99 and out["xgmi_GB"] > prev["xgmi_GB"]
        prev = out


def test_model_dag_matches_runtime_simulation(tmp_path):
    """The runtime's own simulation mode (runtime_simulation=1) on the
    ptgpp-compiled dpotrf_L.jdf with its SIMCOST (costs of a 1024-tile run,
    PARSEC_SIMCOST_NB, on small real tiles) yields exactly the longest path the
    model computes for the same DAG and costs."""
    import subprocess
    import sys

    NT = 12
    code = f"""
import numpy as np, parsec_amd as pa
pa.mca_set("runtime_simulation", "1")
ctx = pa.init(4)
nb = 8
N = {NT} * nb
A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
S = np.random.default_rng(1).standard_normal((N, N)); S = S @ S.T + N * np.eye(N)
for m in range(A.mt):
    for n in range(A.nt):
        A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
tp, info = pa.dpotrf_jdf_new(A)
ctx.add_taskpool(tp); ctx.start(); ctx.wait()
print("SIMDATE", tp.simulation_date)
ctx.fini()
"""
    env = dict(__import__("os").environ, PARSEC_SIMCOST_NB="1024", PARSEC_MCA_device_hip_enabled="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    date = int(next(l for l in r.stdout.splitlines() if l.startswith("SIMDATE")).split()[1])
    assert date == sm.critical_path_exact_ns(NT, sm.simcost_ns(1024))


def test_serial_receive_queue():
    """Round 5: one serial, priority-ordered receive queue per rank (the code's
    fetch queue over one copy-engine pull stream) with the critical-stream TRSM:
    the graph drains, moves the same bytes as per-link transfers, and the span
    respects both the chain bound and the receive bound (a rank cannot take in
    its tiles faster than one at a time). Priority order can beat per-link FIFO
    links, so the two are not ordered."""
    NT, nb = 16, 1024
    xfer_us = nb * nb * 8 / 50e9 * 1e6
    for r in (2, 4, 8):
        P, Q = sm.grid_of(r)
        link = sm.simulate(NT, nb, P, Q, gemm_tf=66.0, potrf_us=350.0, link_gbs=50.0, lat_us=25.0, recv="per-link", trsm_us=265.0)
        ser = sm.simulate(NT, nb, P, Q, gemm_tf=66.0, potrf_us=350.0, link_gbs=50.0, lat_us=25.0, recv="serial", trsm_us=265.0)
        assert ser["xgmi_GB"] == link["xgmi_GB"]
        chain = sm.critical_path_us(NT, 350.0, 265.0, nb ** 3 / 66e12 * 1e6 / 0.85, xfer_us + 25.0, P, Q)
        assert ser["span_ms"] * 1e3 >= chain * 0.999
        per_rank_tiles = ser["xgmi_GB"] * 1e9 / (nb * nb * 8) / r
        assert ser["span_ms"] * 1e3 >= per_rank_tiles * xfer_us * 0.999


def test_receive_lanes():
    """Round 6: per-source receive lanes issued in multi-source gather waves
    (one tile per source link per wave, the code's fetch-queue lanes and
    flush_gather): same bytes as the other receive models, several sources in
    one wave at 4+ ranks, never slower than one serial receive queue, and the
    receive bound becomes a per-link one."""
    NT, nb = 16, 1024
    xfer_us = nb * nb * 8 / 50e9 * 1e6
    for r in (2, 4, 8):
        P, Q = sm.grid_of(r)
        ser = sm.simulate(NT, nb, P, Q, gemm_tf=66.0, potrf_us=350.0, link_gbs=50.0, lat_us=25.0, recv="serial", trsm_us=265.0)
        lan = sm.simulate(NT, nb, P, Q, gemm_tf=66.0, potrf_us=350.0, link_gbs=50.0, lat_us=25.0, recv="lanes", trsm_us=265.0)
        assert lan["xgmi_GB"] == ser["xgmi_GB"]
        assert lan["span_ms"] <= ser["span_ms"] * 1.001
        chain = sm.critical_path_us(NT, 350.0, 265.0, nb ** 3 / 66e12 * 1e6 / 0.85, xfer_us + 25.0, P, Q)
        assert lan["span_ms"] * 1e3 >= chain * 0.999
        if r >= 4:
            assert lan["max_wave"] >= 2
