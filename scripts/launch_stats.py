"""Per-dispatch duration of one kernel in a rocprofv3 kernel trace, by grid size.
usage: python scripts/launch_stats.py run_kernel_trace.csv KERNEL_SUBSTRING"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    if sys.argv[2] in r["Kernel_Name"]:
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        by[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for g in sorted(by):
    v = sorted(by[g])
    print(f"grid {g:5d}: n={len(v):5d} median {v[len(v) // 2]:8.1f} us  min {v[0]:8.1f}  max {v[-1]:8.1f}")
