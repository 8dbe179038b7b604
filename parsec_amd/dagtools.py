"""DAG tools over the graphs the runtime's grapher writes (`--mca parsec_dot
<base>`, one DOT file per rank) -- the roles of the reference's
tools/dagenum.c (enumerate a recorded DAG: nodes, successors, dependency
check) and tools/grapher.c (dump a taskpool's DAG), plus the per-rank merge.

    python -m parsec_amd.dagtools stats  graph-0.dot [graph-1.dot ...]
    python -m parsec_amd.dagtools levels graph-0.dot ...     # tasks per topological level
    python -m parsec_amd.dagtools classes graph-0.dot ...    # tasks per task class
    python -m parsec_amd.dagtools merge out.dot graph-*.dot

`stats` reports nodes, edges, roots, leaves, the critical path length (in
tasks), the average parallelism (nodes / critical path) and whether the graph
is acyclic (a cycle means a broken dependency specification).
"""
import re
import sys
from collections import Counter, defaultdict, deque

_NODE = re.compile(r'^\s*("?[^\s"\[]+"?)\s*\[label="([^"]*)"')
_EDGE = re.compile(r'^\s*("?[^\s"]+"?)\s*->\s*("?[^\s"\[;]+"?)')


class Dag:
    def __init__(self):
        self.labels = {}
        self.succ = defaultdict(set)
        self.pred = defaultdict(set)

    @property
    def nodes(self):
        return set(self.labels) | set(self.succ) | set(self.pred)

    def edges(self):
        return sum(len(s) for s in self.succ.values())

    def topo_levels(self):
        """Longest-path level of every node (roots = 0); None if cyclic."""
        nodes = self.nodes
        indeg = {n: len(self.pred[n]) for n in nodes}
        level = {n: 0 for n in nodes}
        q = deque(n for n in nodes if indeg[n] == 0)
        seen = 0
        while q:
            n = q.popleft()
            seen += 1
            for s in self.succ[n]:
                level[s] = max(level[s], level[n] + 1)
                indeg[s] -= 1
                if indeg[s] == 0:
                    q.append(s)
        return level if seen == len(nodes) else None

    def stats(self):
        nodes = self.nodes
        levels = self.topo_levels()
        cp = (max(levels.values()) + 1) if levels else None
        return {
            "nodes": len(nodes),
            "edges": self.edges(),
            "roots": sum(1 for n in nodes if not self.pred[n]),
            "leaves": sum(1 for n in nodes if not self.succ[n]),
            "acyclic": levels is not None,
            "critical_path": cp,
            "avg_parallelism": (len(nodes) / cp) if cp else None,
        }

    def class_of(self, n):
        lab = self.labels.get(n, n.strip('"'))
        return lab.split("(")[0]


def read_dot(paths):
    """Parse grapher DOT files (several ranks merge into one DAG)."""
    g = Dag()
    for p in paths:
        with open(p) as f:
            for line in f:
                m = _EDGE.match(line)
                if m:
                    a, b = m.group(1), m.group(2)
                    g.succ[a].add(b)
                    g.pred[b].add(a)
                    continue
                m = _NODE.match(line)
                if m:
                    g.labels[m.group(1)] = m.group(2)
    return g


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) < 2:
        print(__doc__)
        return 1
    cmd = argv.pop(0)
    if cmd == "merge":
        from .profiling import dot_merge

        dot_merge(argv[1:], argv[0])
        return 0
    g = read_dot(argv)
    if cmd == "stats":
        for k, v in g.stats().items():
            print(f"{k:16s} {v}")
        return 0 if g.topo_levels() is not None else 2
    if cmd == "levels":
        lv = g.topo_levels()
        if lv is None:
            print("cycle detected")
            return 2
        for level, n in sorted(Counter(lv.values()).items()):
            print(f"{level:6d} {n}")
        return 0
    if cmd == "classes":
        for c, n in Counter(g.class_of(x) for x in g.nodes).most_common():
            print(f"{c:24s} {n}")
        return 0
    print(__doc__)
    return 1


if __name__ == "__main__":
    sys.exit(main())
