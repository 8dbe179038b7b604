"""Per-edge latency of remote dependencies from the per-rank traces of one run.

For every received flow (COMM_DATA_RCV at the receiver) this joins:
  ACTIVATE  sender: activation handed to the comm engine (COMM_ACTIVATE begin)
  RCV       receiver: activation processed, data requested (eager IPC: pull
            issued at once; otherwise a GET goes back to the sender)
  PULL      receiver: the device copy of the IPC pull, issued -> landed
  RCV end   receiver: flow delivered to the local successors
Clocks: each trace stores its absolute start (steady clock, shared by the
processes of one node), so begin times are comparable across ranks.

usage: python scripts/comm_edges.py <profile_filename prefix> NRANKS
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsec_amd import profiling  # noqa: E402


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))] if v else float("nan")


def main():
    base, n = sys.argv[1], int(sys.argv[2])
    traces = [profiling.read_trace(f"{base}-{r}.prof") for r in range(n)]
    t0 = {tr.rank: tr.t0 for tr in traces}
    rows = profiling.intervals(traces)
    acts = {}
    for r in rows:
        if r["type"] == "COMM_ACTIVATE":
            acts[(r["rank"], r["peer"], r["send_id"])] = r["begin"] + t0[r["rank"]]
    pulls = {(r["rank"], r["event_id"]): r for r in rows if r["type"] == "COMM_IPC_PULL"}
    edges = []
    for r in rows:
        if r["type"] != "COMM_DATA_RCV":
            continue
        rb = r["begin"] + t0[r["rank"]]
        a = acts.get((r["peer"], r["rank"], r["send_id"]))
        p = pulls.get((r["rank"], r["event_id"]))
        e = {"bytes": r["bytes"], "plane": r["plane"], "act": (rb - a) / 1e3 if a else None,
             "rcv_total": r["duration"] / 1e3}
        if p:
            e["to_pull"] = (p["begin"] - r["begin"]) / 1e3
            e["pull"] = p["duration"] / 1e3
            e["after_pull"] = (r["end"] - p["end"]) / 1e3
        edges.append(e)
    print(f"{len(edges)} received flows over {n} ranks ({sum(1 for e in edges if 'pull' in e)} IPC pulls)")
    for k, what in (("act", "activation: sender hand-off -> receiver processed"),
                    ("to_pull", "receiver processed -> IPC pull issued (GET round trip unless eager)"),
                    ("pull", "IPC pull: copy issued -> landed"),
                    ("after_pull", "landed -> delivered to successors"),
                    ("rcv_total", "receiver processed -> delivered")):
        v = [e[k] for e in edges if e.get(k) is not None]
        if not v:
            continue
        print(f"  {k:10s} n={len(v):5d} median {statistics.median(v):8.1f} us  p10 {pct(v, .1):8.1f}  p90 {pct(v, .9):8.1f}  max {max(v):8.1f}   {what}")
    big = [e for e in edges if e.get("pull") and e["bytes"] >= 1 << 20]
    if big:
        bw = [e["bytes"] / (e["pull"] * 1e3) for e in big]
        print(f"  pull bandwidth (>= 1 MiB payloads): median {statistics.median(bw):.1f} GB/s over {len(big)} pulls")


if __name__ == "__main__":
    main()
