"""Per-panel critical chain of a DPOTRF run from a rocprofv3 kernel trace.

POTRF(k) of an nb-tile is a run of tile-POTRF kernels on the critical queue
(dpotrf_step_kernel: nb/64 + 1 launches; legacy: nb/64 dpotrf_diag_inv plus
the TRSM/GEMM pieces between them). For the LAST factorization in the trace
(factorizations are separated by > 2 ms of silence) this prints, per panel k:
  potrf  = first tile-POTRF kernel start -> last one's end (incl. waiting for CUs)
  queued = time inside that span with a POTRF kernel dispatched but not running
  chain  = POTRF(k) start -> POTRF(k+1) start (TRSM + SYRK + hops)
usage: python scripts/critical_chain.py run_kernel_trace.csv NB [N]
"""
import csv
import sys

path, nb = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows if "parsec::kern" in r["Kernel_Name"])
steps, cur = [], [ks[0]]
for k in ks[1:]:
    if k[0] - max(c[1] for c in cur[-50:]) > 2_000_000:
        steps.append(cur)
        cur = []
    cur.append(k)
steps.append(cur)
st = steps[-1]
t0 = st[0][0]
step_kernel = any("dpotrf_step_kernel" in n for _, _, n, _ in st)
per = nb // 64 + 1 if step_kernel else nb // 64
key = "dpotrf_step_kernel" if step_kernel else "dpotrf_diag_inv"
pk = [k for k in st if key in k[2]]
# the silence between factorizations can be short: with N given, keep the last
# NT tile POTRFs (the last factorization) counted from the end
if len(sys.argv) > 3:
    NT = (int(sys.argv[3]) + nb - 1) // nb
    pk = [k for k in ks if key in k[2]][-NT * per:]
    t0 = pk[0][0]
    st = [k for k in ks if k[0] >= t0]
groups = [pk[i:i + per] for i in range(0, len(pk), per)]
print(f"factorization span {(max(k[1] for k in st) - t0) / 1e3:.1f} us, {len(groups)} panels, tile POTRF = {per} x {key}")
print(f"{'k':>3} {'start':>9} {'potrf':>8} {'chain':>8}")
tot_p = tot_c = 0.0
for i, g in enumerate(groups):
    s, e = g[0][0], max(x[1] for x in g)
    nxt = groups[i + 1][0][0] if i + 1 < len(groups) else None
    chain = (nxt - s) / 1e3 if nxt else float("nan")
    tot_p += (e - s) / 1e3
    if nxt:
        tot_c += chain
    print(f"{i:3d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {chain:8.1f}")
print(f"sum potrf {tot_p / 1e3:.2f} ms, sum chain {tot_c / 1e3:.2f} ms")
