"""What the critical queue runs between two tile POTRFs (config-2 chain anatomy).

From a rocprofv3 --kernel-trace CSV of a DPOTRF run, take the last
factorization (the last NT tile POTRFs), find the queue the tile-POTRF kernels
run on, and for every panel k split the window POTRF(k) end -> POTRF(k+1)
start into the kernels that queue ran (by kind, with workgroup counts) and the
idle time where nothing ran on it (host hop: completion poll, release,
dispatch). Prints a per-panel table and the totals.
usage: python scripts/chain_window.py run_kernel_trace.csv NB N
"""
import collections
import csv
import sys

path, nb, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
NT = (N + nb - 1) // nb
rows = list(csv.DictReader(open(path)))


def wgs(r):
    try:
        g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        w = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
        return g // max(w, 1)
    except ValueError:
        return 0


def kind(name):
    for key, k in (("dpotrf_step_kernel", "potrf"), ("trsm_w", "trsm_w"), ("dtrsm_inv", "trsm_inv"), ("unpack", "unpack"),
                   ("dgemm_batch_kernel", "gemm"), ("copy", "copy"), ("memset", "memset"), ("fill", "memset")):
        if key in name:
            return k
    return name.split("(")[0][-30:]


ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"], wgs(r)) for r in rows
            if "parsec::kern" in r["Kernel_Name"] or "__amd_rocclr" in r["Kernel_Name"])
per = nb // 64 + 1
pk = [k for k in ks if "dpotrf_step_kernel" in k[2]][-NT * per:]
crit_q = collections.Counter(k[3] for k in pk).most_common(1)[0][0]
t0 = pk[0][0]
groups = [pk[i:i + per] for i in range(0, len(pk), per)]
crit = [k for k in ks if k[3] == crit_q and k[0] >= t0]
tot = collections.defaultdict(float)
tot_wg = collections.defaultdict(list)
print(f"critical queue {crit_q}; {len(groups)} panels; times in us")
print(f"{'k':>3} {'potrf':>7} {'window':>7} {'idle':>7}  kernels in the window (kind x wgs: us)")
sum_idle = sum_win = sum_potrf = 0.0
for i in range(len(groups) - 1):
    ps, pe = groups[i][0][0], max(x[1] for x in groups[i])
    ns = groups[i + 1][0][0]
    win = [k for k in crit if k[0] >= pe and k[1] <= ns and "dpotrf_step_kernel" not in k[2]]
    busy, last = 0.0, pe
    for k in win:
        s = max(k[0], last)
        if k[1] > s:
            busy += k[1] - s
        last = max(last, k[1])
    idle = (ns - pe) - busy
    sum_idle += idle
    sum_win += ns - pe
    sum_potrf += pe - ps
    desc = []
    for k in win:
        kd = kind(k[2])
        tot[kd] += (k[1] - k[0]) / 1e3
        tot_wg[kd].append(k[4])
        desc.append(f"{kd}x{k[4]}:{(k[1] - k[0]) / 1e3:.0f}")
    if i < 6 or i % 8 == 0 or i >= len(groups) - 3:
        print(f"{i:3d} {(pe - ps) / 1e3:7.1f} {(ns - pe) / 1e3:7.1f} {idle / 1e3:7.1f}  {' '.join(desc)}")
print(f"sum potrf {sum_potrf / 1e6:.2f} ms, sum windows {sum_win / 1e6:.2f} ms, of which critical queue idle {sum_idle / 1e6:.2f} ms")
for kd, v in sorted(tot.items(), key=lambda x: -x[1]):
    w = tot_wg[kd]
    print(f"  {kd:10s} {v / 1e3:8.2f} ms in {len(w)} launches, wgs median {sorted(w)[len(w) // 2]}")
