"""Mean per dispatch of every PMC counter of the kernels whose name contains a
pattern, from a rocprofv3 --pmc --output-format csv counter_collection.csv.
usage: python scripts/pmc_summary.py run_counter_collection.csv dgemm_batch_kernel"""
import collections
import csv
import sys

path, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(float)
disp = collections.defaultdict(set)
names = set()
for r in csv.DictReader(open(path)):
    if pat not in r["Kernel_Name"]:
        continue
    names.add(r["Kernel_Name"][:110])
    vals[r["Counter_Name"]] += float(r["Counter_Value"])
    disp[r["Counter_Name"]].add(r["Dispatch_Id"])
print(f"== {path}")
for n in sorted(names):
    print(f"   kernel {n}")
for c in sorted(vals):
    print(f"   {c:28s} {vals[c] / max(1, len(disp[c])):.4e}   ({len(disp[c])} dispatches)")
