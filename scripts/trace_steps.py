"""Split a rocprofv3 kernel trace of bench.py into factorization steps (runs of
parsec::kern kernels separated by > 2 ms of silence) and report, per step: span,
GPU busy fraction, time in each kernel family, and the sum of the critical-path
launches (tile POTRF pieces)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")) for r in rows if "parsec::kern" in r["Kernel_Name"])
steps, cur = [], [ks[0]]
for k in ks[1:]:
    if k[0] - max(c[1] for c in cur[-50:]) > 2_000_000:
        steps.append(cur)
        cur = []
    cur.append(k)
steps.append(cur)


def fam(n):
    for key in ("dgemm_batch_kernel<128", "dgemm_batch_kernel<64", "dpotrf_diag", "dtrsm_inv", "copy_tiles", "qr_", "stencil", "copy_bytes"):
        if key in n:
            return key
    return n[:40]


for i, st in enumerate(steps):
    t0, t1 = st[0][0], max(k[1] for k in st)
    ev = sorted([(s, 1) for s, *_ in st] + [(e, -1) for _, e, *_ in st])
    c, last, busy = 0, ev[0][0], 0
    for t, d in ev:
        if c > 0:
            busy += t - last
        c += d
        last = t
    by = collections.Counter()
    for s, e, n, q in st:
        by[fam(n)] += e - s
    qs = collections.Counter(q for *_, q in st)
    print(f"step {i}: {len(st)} kernels, span {(t1 - t0) / 1e6:.2f} ms, busy {busy / (t1 - t0):.1%}, queues {len(qs)}")
    for f, v in by.most_common(8):
        print(f"    {f:28s} {v / 1e6:8.2f} ms")
