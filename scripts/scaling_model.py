"""Discrete-event MODEL of tiled DPOTRF (lower) on 1/2/4/8 MI355X ranks.

This is a PREDICTION tool, not a measurement: the driver's 8-GPU node is the
only place the multi-GPU numbers can be measured (every gpurun box has one
GPU). It replays the task graph the runtime executes (csrc/algos/jdf/dpotrf_L.jdf,
reference dplasma zpotrf_L.jdf) on a model of the machine:

  * one rank per GPU, tile (m, n) on rank (m % P) * Q + (n % Q) of a P x Q grid
    (bench.py grid_of; reference two_dim_rectangle_cyclic.c rank_of);
  * per GPU a BULK server that runs TRSM / SYRK / GEMM one after another in
    task-priority order at the measured grouped-GEMM rate (a fluid model of the
    2 bulk streams: the GPU is throughput-shared, so serial-at-full-rate gives
    the same completion profile), and a CRITICAL lane for POTRF(k) with the
    measured tile-POTRF latency under load (it runs beside bulk work on the
    critical stream, profiles/r4_chain*.txt);
  * a tile produced on rank r and read by tasks on rank s != r crosses the
    (r, s) xGMI link ONCE (the runtime's per-rank activation aggregation), after
    a per-message latency. Round 6 (what the code does, `--recv lanes`): every
    rank queues its inbound pulls per SOURCE rank (csrc/comm/fetch_queue.hpp
    lanes, priority ordered by the consuming task's priority) and issues them in
    multi-source gather launches on its one copy stream (shm_engine.cpp
    flush_gather): a launch moves the head tile of every source with work at
    once, one per xGMI link, and the next launch follows it. `--recv serial` is
    round 5 (one pull at a time per rank), `--recv per-link` round 4 (one
    transfer at a time per directed link, no wave synchronization);
  * the panel chain's TRSM(k+1, k) / SYRK(k, k+1) run on the critical stream
    with a measured latency (`--trsm-us`: the critical 64x64 grouped TRSM
    W-GEMM averages 265 us under load at config 3, profiles/r5_kernel_stats_c3_v1.csv).

Calibration: --gemm-tf is the sustained bulk rate; the 1-rank prediction is
compared with the measured 1-GPU number (BENCH json) so the residual model error
is visible next to the prediction.

usage: python scripts/scaling_model.py [--n 65536 --nb 1024] [--gemm-tf 66]
       [--potrf-us 520] [--link-gbs 50] [--lat-us 25] [--ranks 1 2 4 8]
"""
import argparse
import heapq
import itertools


def grid_of(n):
    # bench.py grid_of: the most square P x Q with P >= Q
    best = (n, 1)
    for q in range(1, n + 1):
        if n % q == 0 and n // q >= q:
            best = (n // q, q)
    return best


def simulate(NT, nb, P, Q, gemm_tf, potrf_us, link_gbs, lat_us, syrk_eff=0.85, trsm_eff=1.0, recv="per-link", trsm_us=None):
    R = P * Q

    def owner(m, n):
        return (m % P) * Q + (n % Q)

    g_us = 2.0 * nb ** 3 / (gemm_tf * 1e12) * 1e6
    cost = {"POTRF": potrf_us, "TRSM": g_us / trsm_eff, "SYRK": g_us / 2 / syrk_eff, "GEMM": g_us}
    xfer_us = nb * nb * 8 / (link_gbs * 1e9) * 1e6 + lat_us

    # ---- task graph: name -> (rank, kind, priority, successors); deps counted
    tasks, nd = {}, {}

    def add(t, rank, kind, prio):
        tasks[t] = (rank, kind, prio, [])
        nd.setdefault(t, 0)

    def dep(a, b):
        tasks[a][3].append(b)
        nd[b] = nd.get(b, 0) + 1

    for k in range(NT):
        # priorities of dpotrf_L.jdf: the panel chain first, then by k
        add(("POTRF", k), owner(k, k), "POTRF", (1 << 30) - k)
        for m in range(k + 1, NT):
            add(("TRSM", m, k), owner(m, k), "TRSM", (1 << 29) - k * NT + (NT - m) if m == k + 1 else (1 << 28) - k * NT - m)
            add(("SYRK", k, m), owner(m, m), "SYRK", (1 << 29) - k if m == k + 1 else (1 << 27) - k * NT - m)
            for n in range(k + 1, m):
                add(("GEMM", m, n, k), owner(m, n), "GEMM", ((1 << 27) if n == k + 1 else 0) - k * NT * NT - m * NT - n)
    for k in range(NT):
        if k > 0:
            dep(("SYRK", k - 1, k), ("POTRF", k))
        for m in range(k + 1, NT):
            dep(("POTRF", k), ("TRSM", m, k))
            if k > 0:
                dep(("GEMM", m, k, k - 1), ("TRSM", m, k))
            dep(("TRSM", m, k), ("SYRK", k, m))
            if k > 0:
                dep(("SYRK", k - 1, m), ("SYRK", k, m))
            for n in range(k + 1, m):
                dep(("TRSM", m, k), ("GEMM", m, n, k))
                dep(("TRSM", n, k), ("GEMM", m, n, k))
                if k > 0:
                    dep(("GEMM", m, n, k - 1), ("GEMM", m, n, k))

    # ---- event simulation
    seq = itertools.count()
    ev = []  # (time, seq, kind, payload)
    bulk_q = [[] for _ in range(R)]
    crit_q = [[] for _ in range(R)]
    bulk_busy = [False] * R
    crit_busy = [False] * R
    link_free = {}  # (src, dst) -> time the link is free
    arrived = {}  # (producer, dst rank) -> arrival time (None: in flight)
    waiting = {}  # (producer, dst rank) -> [successors waiting for that tile]
    busy_us = [0.0] * R
    bytes_sent = 0
    now = 0.0

    def on_crit(t):
        # the panel chain on the critical stream: POTRF, and with a measured
        # chain latency also TRSM(k+1, k) and SYRK(k, k+1)
        kind = tasks[t][1]
        if kind == "POTRF":
            return True
        if trsm_us is None:
            return False
        return (kind == "TRSM" and t[1] == t[2] + 1) or (kind == "SYRK" and t[2] == t[1] + 1)

    def crit_cost(t):
        kind = tasks[t][1]
        return cost["POTRF"] if kind == "POTRF" else trsm_us if kind == "TRSM" else cost["SYRK"]

    recv_q = [[] for _ in range(R)]  # serial receive: (-prio, seq, key)
    lane_q = [{} for _ in range(R)]  # lanes: source rank -> [(-prio, seq, key)]
    recv_busy = [False] * R
    max_wave = [0] * R

    def recv_kick(r, at):
        if recv_busy[r]:
            return
        if recv == "lanes":
            wave = [heapq.heappop(q)[2] for q in lane_q[r].values() if q]
            if not wave:
                return
            recv_busy[r] = True
            max_wave[r] = max(max_wave[r], len(wave))
            heapq.heappush(ev, (at + xfer_us - lat_us, next(seq), "wave", (r, wave)))
            return
        if not recv_q[r]:
            return
        _, _, key = heapq.heappop(recv_q[r])
        recv_busy[r] = True
        heapq.heappush(ev, (at + xfer_us - lat_us, next(seq), "arrive", key))

    def ready(t, at):
        rank, kind, prio, _ = tasks[t]
        q = crit_q[rank] if on_crit(t) else bulk_q[rank]
        heapq.heappush(q, (-prio, next(seq), t))
        heapq.heappush(ev, (at, next(seq), "kick", rank))

    def satisfy(t, at):
        nd[t] -= 1
        if nd[t] == 0:
            ready(t, at)

    def kick(rank, at):
        if not crit_busy[rank] and crit_q[rank]:
            _, _, t = heapq.heappop(crit_q[rank])
            crit_busy[rank] = True
            heapq.heappush(ev, (at + crit_cost(t), next(seq), "done", (t, "crit")))
        if not bulk_busy[rank] and bulk_q[rank]:
            _, _, t = heapq.heappop(bulk_q[rank])
            bulk_busy[rank] = True
            c = cost[tasks[t][1]]
            busy_us[rank] += c
            heapq.heappush(ev, (at + c, next(seq), "done", (t, "bulk")))

    for t in tasks:
        if nd[t] == 0:
            ready(t, 0.0)
    finish = 0.0
    while ev:
        now, _, kind, p = heapq.heappop(ev)
        if kind == "kick":
            kick(p, now)
        elif kind == "done":
            t, lane = p
            rank = tasks[t][0]
            if lane == "crit":
                crit_busy[rank] = False
            else:
                bulk_busy[rank] = False
            finish = max(finish, now)
            for s in tasks[t][3]:
                sr = tasks[s][0]
                if sr == rank:
                    satisfy(s, now)
                    continue
                key = (t, sr)
                if key in arrived:
                    if arrived[key] is None:
                        waiting[key].append(s)
                    else:
                        satisfy(s, now)
                    continue
                # one transfer of the tile to that rank
                arrived[key] = None
                waiting[key] = [s]
                bytes_sent += nb * nb * 8
                if recv in ("serial", "lanes"):
                    # the activation reaches the receiver after the message
                    # latency; its pull then queues behind the rank's other pulls
                    heapq.heappush(ev, (now + lat_us, next(seq), "request", (key, tasks[s][2])))
                    continue
                start = max(now, link_free.get((rank, sr), 0.0))
                link_free[(rank, sr)] = start + xfer_us - lat_us
                heapq.heappush(ev, (start + xfer_us, next(seq), "arrive", key))
            kick(rank, now)
        elif kind == "request":
            key, prio = p
            if recv == "lanes":
                heapq.heappush(lane_q[key[1]].setdefault(tasks[key[0]][0], []), (-prio, next(seq), key))
            else:
                heapq.heappush(recv_q[key[1]], (-prio, next(seq), key))
            recv_kick(key[1], now)
        elif kind == "wave":
            r, wave = p
            recv_busy[r] = False
            for key in wave:
                arrived[key] = now
                for s in waiting.pop(key):
                    satisfy(s, now)
            recv_kick(r, now)
        elif kind == "arrive":
            arrived[p] = now
            if recv == "serial":
                recv_busy[p[1]] = False
                recv_kick(p[1], now)
            for s in waiting.pop(p):
                satisfy(s, now)
    assert all(v == 0 for v in nd.values()), "graph did not drain"
    n = NT * nb
    flops = n ** 3 / 3.0
    return {"ranks": R, "grid": f"P{P}xQ{Q}", "span_ms": finish / 1e3, "tflops": flops / (finish * 1e-6) / 1e12,
            "bulk_util": sum(busy_us) / (R * finish), "xgmi_GB": bytes_sent / 1e9, "max_wave": max(max_wave)}


def critical_path_exact_ns(NT, costs_ns):
    """Longest path of the DPOTRF DAG with per-kind task costs (ns; no
    communication, infinite GPUs): what the runtime's simulation mode computes
    for csrc/algos/jdf/dpotrf_L.jdf with its SIMCOST (runtime_simulation=1)."""
    done = {}
    for k in range(NT):
        p_in = done.get(("SYRK", k - 1, k), 0)
        done[("POTRF", k)] = p_in + costs_ns["POTRF"]
        for m in range(k + 1, NT):
            t_in = max(done[("POTRF", k)], done.get(("GEMM", m, k, k - 1), 0))
            done[("TRSM", m, k)] = t_in + costs_ns["TRSM"]
        for m in range(k + 1, NT):
            s_in = max(done[("TRSM", m, k)], done.get(("SYRK", k - 1, m), 0))
            done[("SYRK", k, m)] = s_in + costs_ns["SYRK"]
            for n in range(k + 1, m):
                g_in = max(done[("TRSM", m, k)], done[("TRSM", n, k)], done.get(("GEMM", m, n, k - 1), 0))
                done[("GEMM", m, n, k)] = g_in + costs_ns["GEMM"]
    return max(done.values())


def simcost_ns(nb, gemm_tf=66.0, potrf_us=None):
    """The per-kind costs of dpotrf_L.jdf's SIMCOST (jdf_simcost), integer ns."""
    g = 2.0 * nb ** 3 / (gemm_tf * 1e3)
    return {"POTRF": int((potrf_us if potrf_us else 520.0 * nb / 1024.0) * 1e3), "TRSM": int(g), "SYRK": int(g / 2 / 0.85), "GEMM": int(g)}


def critical_path_us(NT, potrf_us, trsm_us, syrk_us, xfer_us, P, Q):
    # lower bound of the span ("chain ms"): POTRF(k) -> TRSM(k+1,k) ->
    # SYRK(k,k+1) -> POTRF(k+1) with infinite GPUs; tile (k,k) -> (k+1,k)
    # changes grid row (a hop when P > 1), (k+1,k) -> (k+1,k+1) changes grid
    # column (a hop when Q > 1)
    hops = (P > 1) + (Q > 1)
    return NT * potrf_us + (NT - 1) * (trsm_us + syrk_us + hops * xfer_us)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=1024)
    ap.add_argument("--gemm-tf", type=float, default=66.0, help="sustained bulk GEMM rate per GPU (TF)")
    ap.add_argument("--potrf-us", type=float, default=520.0, help="tile POTRF latency under load (us)")
    ap.add_argument("--link-gbs", type=float, nargs="+", default=[50.0], help="effective GB/s per directed xGMI peer link")
    ap.add_argument("--lat-us", type=float, default=25.0, help="per-message latency (activation + pull setup)")
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--measured-1gpu-tf", type=float, default=None)
    ap.add_argument("--recv", choices=["lanes", "serial", "per-link"], default="lanes", help="inbound transfers: per-source lanes in gather waves (the code, round 6), one serial queue per rank (round 5) or one per directed link (round 4)")
    ap.add_argument("--trsm-us", type=float, default=265.0, help="TRSM(k+1,k) latency on the critical stream (us); <0: in the bulk at the GEMM rate")
    a = ap.parse_args()
    NT = a.n // a.nb
    trsm = a.trsm_us if a.trsm_us >= 0 else None
    print(f"MODEL PREDICTION (not a measurement): DPOTRF N={a.n} nb={a.nb} ({NT}x{NT} tiles), bulk GEMM {a.gemm_tf} TF/GPU, "
          f"tile POTRF {a.potrf_us} us, TRSM(k+1,k) {a.trsm_us} us, message latency {a.lat_us} us, receive {a.recv}")
    for bw in a.link_gbs:
        print(f"-- xGMI effective {bw} GB/s per directed peer link")
        print(f"{'ranks':>5} {'grid':>6} {'span ms':>9} {'TF (job)':>9} {'TF/GPU':>7} {'eff':>5} {'bulk util':>9} {'xGMI GB':>8} {'chain ms':>8} {'max wave':>8}")
        base = None
        for r in a.ranks:
            P, Q = grid_of(r)
            out = simulate(NT, a.nb, P, Q, a.gemm_tf, a.potrf_us, bw, a.lat_us, recv=a.recv, trsm_us=trsm)
            base = base or out["tflops"]
            eff = out["tflops"] / (base * r)
            g_us = 2.0 * a.nb ** 3 / (a.gemm_tf * 1e12) * 1e6
            chain = critical_path_us(NT, a.potrf_us, trsm if trsm is not None else g_us, g_us / 2 / 0.85, a.nb * a.nb * 8 / (bw * 1e9) * 1e6 + a.lat_us, P, Q) / 1e3
            print(f"{r:>5} {out['grid']:>6} {out['span_ms']:>9.1f} {out['tflops']:>9.1f} {out['tflops'] / r:>7.1f} {eff:>5.2f} {out['bulk_util']:>9.2f} {out['xgmi_GB']:>8.1f} {chain:>8.1f} {out['max_wave']:>8}")
    if a.measured_1gpu_tf:
        P, Q = grid_of(1)
        one = simulate(NT, a.nb, P, Q, a.gemm_tf, a.potrf_us, a.link_gbs[0], a.lat_us, recv=a.recv, trsm_us=trsm)
        print(f"calibration: model 1-GPU {one['tflops']:.1f} TF vs measured {a.measured_1gpu_tf:.1f} TF ({(one['tflops'] / a.measured_1gpu_tf - 1) * 100:+.1f} %)")


if __name__ == "__main__":
    main()
