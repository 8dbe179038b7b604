"""Copy-engine occupancy from a rocprofv3 memory-copy trace (CSV): per
direction the number of copies, bytes, summed copy time and the union of the
copy intervals; occupancy = busy (union) / span, where span runs from the
first to the last copy. Overlapping copies (several engines at once) make the
summed time exceed the union.

usage: python scripts/copy_occupancy.py <..._memory_copy_trace.csv>
"""
import csv
import sys
from collections import defaultdict


def col(row, *names):
    for n in names:
        for k in row:
            if k.lower() == n.lower():
                return row[k]
    for n in names:
        for k in row:
            if n.lower() in k.lower():
                return row[k]
    return None


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    if not rows:
        print("no copies")
        return
    by = defaultdict(list)
    allv = []
    for r in rows:
        s, e = int(col(r, "Start_Timestamp", "start")), int(col(r, "End_Timestamp", "end"))
        d = col(r, "Direction", "Kind") or "?"
        b = col(r, "Bytes", "Size") or "0"
        by[d].append((s, e, int(b) if str(b).isdigit() else 0))
        allv.append((s, e))
    t0, t1 = min(s for s, _ in allv), max(e for _, e in allv)
    span = t1 - t0
    print(f"copies={len(allv)} span_ms={span / 1e6:.1f} busy_union_ms={union(allv) / 1e6:.1f} occupancy={union(allv) / span:.3f}")
    for d, v in sorted(by.items()):
        tb = sum(x[2] for x in v)
        st = sum(e - s for s, e, _ in v)
        print(f"  {d}: n={len(v)} MiB={tb >> 20} sum_ms={st / 1e6:.1f} union_ms={union([(s, e) for s, e, _ in v]) / 1e6:.1f} "
              f"GB/s(sum)={tb / max(st, 1):.2f}")


if __name__ == "__main__":
    main()
