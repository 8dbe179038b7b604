"""Summarise a rocprofv3 kernel trace: per kernel, grid-size histogram, and the
fraction of wall time with >= 2 kernels in flight (last timed region only)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), int(r.get("Workgroup_Size_X", 1) or 1), r.get("Stream_Id", r.get("Queue_Id", ""))))
ks.sort()
# last half of the run = the timed step
t0, t1 = ks[0][0], max(k[1] for k in ks)
mid = ks[len(ks) // 2][0]
sel = [k for k in ks if k[0] >= mid]
by = collections.defaultdict(list)
for s, e, n, g, wg, st in sel:
    by[n].append((e - s, g // max(wg, 1)))
for n, v in sorted(by.items(), key=lambda x: -sum(d for d, _ in x[1])):
    wgs = collections.Counter(g for _, g in v)
    print(f"{n:50s} n={len(v):5d} tot={sum(d for d,_ in v)/1e6:8.2f} ms avg={sum(d for d,_ in v)/len(v)/1e3:8.1f} us  WGs={dict(wgs.most_common(6))}")
# concurrency
ev = []
for s, e, *_ in sel:
    ev += [(s, 1), (e, -1)]
ev.sort()
cur, last, busy, multi = 0, ev[0][0], 0, 0
for t, d in ev:
    if cur >= 1: busy += t - last
    if cur >= 2: multi += t - last
    cur += d; last = t
span = ev[-1][0] - ev[0][0]
print(f"span {span/1e6:.1f} ms, GPU busy {busy/span:.1%}, >=2 kernels {multi/span:.1%}; streams {collections.Counter(k[5] for k in sel).most_common(8)}")
