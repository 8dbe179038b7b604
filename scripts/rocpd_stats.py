"""Summaries of a rocprofv3 rocpd database (ROCm 7 default output, *_results.db):
top kernels, per-queue busy time, and idle gaps of the union of kernels inside
the last window of a run (the timed factorizations).

    python scripts/rocpd_stats.py gpurun_out/s2/p16/run_results.db [--window-ms 40] [--top 15]
"""
import argparse
import sqlite3


def short(name, n=90):
    name = name.replace("parsec::kern::", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--window-ms", type=float, default=0.0, help="also analyse the last W ms of kernel activity (0: skip)")
    ap.add_argument("--match", default="parsec", help="window analysis: only kernels whose name contains this")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels order by total_duration desc").fetchall()
    print(f"# top kernels of {a.db} (whole run)")
    for name, calls, tot, avg, pct in rows[:a.top]:
        # top_kernels reports microseconds
        print(f"{short(name):92s} calls={calls:7d} total_ms={tot / 1e3:9.2f} avg_us={avg:8.1f} pct={pct:5.1f}")
    if a.window_ms <= 0:
        return
    ks = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    ks = [k for k in ks if a.match in k[0]]
    if not ks:
        return
    t_end = max(k[2] for k in ks)
    t0 = t_end - a.window_ms * 1e6
    win = [k for k in ks if k[2] > t0]
    t_start = min(k[1] for k in win)
    span = t_end - t_start
    # union of busy intervals
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for _, s, e, _ in sorted(win, key=lambda k: k[1]):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps.sort()
    med = gaps[len(gaps) // 2] if gaps else 0
    print(f"# window: last {span / 1e6:.2f} ms of '{a.match}' kernels: {len(win)} dispatches, busy {busy / span * 100:.1f}%, "
          f"idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps (median {med / 1e3:.1f} us, max {gaps[-1] / 1e3 if gaps else 0:.1f} us)")
    per = {}
    for name, s, e, q in win:
        p = per.setdefault(short(name, 70), [0, 0])
        p[0] += 1
        p[1] += e - s
    for name, (n, tot) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {name:72s} n={n:6d} sum_ms={tot / 1e6:8.2f} ({tot / span * 100:5.1f}% of span)")
    perq = {}
    for name, s, e, q in win:
        perq[q] = perq.get(q, 0) + e - s
    print("  per-queue kernel time: " + ", ".join(f"q{q} {t / 1e6:.2f} ms" for q, t in sorted(perq.items())))


if __name__ == "__main__":
    main()
