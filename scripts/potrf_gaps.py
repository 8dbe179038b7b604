"""Tile-POTRF step kernels of a DPOTRF rocprofv3 kernel trace: per POTRF (nb/64 + 1
consecutive dpotrf_step_kernel launches on the critical queue), the time the
step kernels ran (sum of their durations) and the gaps between them (launch /
dispatch latency, waiting for a CU) -- the last factorization of the trace.
usage: python scripts/potrf_gaps.py run_kernel_trace.csv NB N"""
import csv
import sys

path, nb, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = list(csv.DictReader(open(path)))
per = nb // 64 + 1
NT = (N + nb - 1) // nb
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "dpotrf_step_kernel" in r["Kernel_Name"])
pk = ks[-NT * per:]  # every tile POTRF is nb/64 + 1 step launches (the last one too)
groups = [pk[i:i + per] for i in range(0, len(pk), per)]
print(f"{len(groups)} tile POTRFs x {per} step kernels (last factorization)")
print(f"{'k':>3} {'span':>8} {'run':>8} {'gaps':>8} {'max_gap':>8}")
ts = tr = 0.0
for i, g in enumerate(groups):
    span = (g[-1][1] - g[0][0]) / 1e3
    run = sum(e - s for s, e in g) / 1e3
    gaps = [(g[j + 1][0] - g[j][1]) / 1e3 for j in range(len(g) - 1)]
    ts += span
    tr += run
    print(f"{i:3d} {span:8.1f} {run:8.1f} {span - run:8.1f} {max(gaps):8.1f}")
print(f"total span {ts / 1e3:.2f} ms, step kernels running {tr / 1e3:.2f} ms, between launches {(ts - tr) / 1e3:.2f} ms")
