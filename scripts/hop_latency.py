"""Host hops on the critical stream from ONE run with both a rocprofv3 kernel
trace and the manager launch log (device_hip_trace_launches=1): for every
retired stream-0 group, notice = manager retire time (R) - end of the last
critical-queue kernel before it, dispatch = next stream-0 launch (L) - R,
start = first kernel start after that L - L. The two clocks (rocprofv3,
steady_clock) are aligned by the smallest L -> kernel-start gap, so every value
is relative to the fastest launch seen (>= 0).
usage: python scripts/hop_latency.py kernel_trace.csv launch.log.gz"""
import bisect
import collections
import csv
import gzip
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows if "parsec::kern" in r["Kernel_Name"])
crit_q = collections.Counter(k[2] for k in ks if "dpotrf_step_kernel" in k[3]).most_common(1)[0][0]
crit = [k for k in ks if k[2] == crit_q]
starts = [k[0] for k in crit]
ends = sorted(k[1] for k in crit)
ev = []
for l in gzip.open(sys.argv[2], "rt"):
    m = re.match(r"\[engine\] t=(\d+) (\w) (stream )?(\d+)", l)
    if m and m.group(2) in "LR" and m.group(4) == "0":
        ev.append((int(m.group(1)) * 1000, m.group(2)))  # us -> ns
launches = [t for t, k in ev if k == "L"]
# clock offset: kernel start - launch time, smallest over launches whose next kernel start is found
gaps = []
for t in launches:
    i = bisect.bisect_left(starts, t - 10**9)
    pass
# align by matching the i-th critical kernel after each launch in order: use the smallest positive (start - L) over a grid of offsets
def first_start_after(t):
    i = bisect.bisect_left(starts, t)
    return starts[i] if i < len(starts) else None
# search offset d so that kernel_time = host_time + d; choose d maximizing matched launches with 0 <= start - (L + d) < 20us
best = None
cands = [s - l for l in launches[:200] for s in starts[:400] if abs((s - l) - (starts[0] - launches[0])) < 5 * 10**8]
cands.sort()
for d in cands[:: max(1, len(cands) // 4000)]:
    hits = 0
    for l in launches[:300]:
        s = first_start_after(l + d)
        if s is not None and s - (l + d) < 20000:
            hits += 1
    if best is None or hits > best[0]:
        best = (hits, d)
d = best[1]
notice, dispatch, start = [], [], []
for idx, (t, k) in enumerate(ev):
    if k != "R":
        continue
    tr = t + d
    j = bisect.bisect_right(ends, tr) - 1
    if j >= 0 and tr - ends[j] < 5 * 10**6:
        notice.append((tr - ends[j]) / 1e3)
    nxt = next((t2 for t2, k2 in ev[idx + 1:] if k2 == "L"), None)
    if nxt is not None:
        dispatch.append((nxt - t) / 1e3)
        s = first_start_after(nxt + d)
        if s is not None:
            start.append((s - (nxt + d)) / 1e3)
def q(v):
    v = sorted(v)
    return f"n={len(v)} median {statistics.median(v):7.1f} us  p90 {v[int(0.9 * (len(v) - 1))]:7.1f} us  sum {sum(v) / 1e3:7.2f} ms"
print(f"clock alignment: {best[0]} of {min(300, len(launches))} launches matched within 20 us")
print("kernel end -> manager notices the group retired:", q(notice))
print("retired -> next stream-0 group launched       :", q(dispatch))
print("launched -> its first kernel starts (rel.)     :", q(start))
