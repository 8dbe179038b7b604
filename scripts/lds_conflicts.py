"""Per-kernel LDS bank-conflict share from a rocprofv3 --pmc SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE counter-collection CSV: extra conflict cycles / all LDS-array
cycles, summed over each kernel's dispatches.
usage: python scripts/lds_conflicts.py run_counter_collection.csv"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:90]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_LDS_IDX_ACTIVE":
        n[k] += 1
rows = []
for k, c in acc.items():
    act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    bc = c.get("SQ_LDS_BANK_CONFLICT", 0.0)
    rows.append((act, bc, k))
for act, bc, k in sorted(rows, reverse=True)[:14]:
    print(f"{k:90s} dispatches={n[k]:6d} lds_cycles={act:12.4g} conflict={bc:12.4g} ({100 * bc / act if act else 0:5.1f} %)")
