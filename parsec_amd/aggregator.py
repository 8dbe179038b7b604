"""Live view of a running application's properties (the role of the
reference's tools/aggregator_visu: read the properties dictionary published
in shared memory while the runtime executes), in text mode.

The runtime publishes when started with ``--mca profile_properties_shm <name>``
(refresh period ``profile_properties_period_ms``, default 100 ms): device
counters, communication counters, user properties (``pa.properties_set``).

    python -m parsec_amd.aggregator <name> [--interval 0.5] [--count N]
"""
import argparse
import os
import re
import sys
import time

_P = re.compile(r'<p name="([^"]*)" value="([^"]*)"/>')
_SEQ = re.compile(r'<properties seq="(\d+)"')


def read(name):
    """(seq, {name: value}) from the shm segment, or None when absent."""
    path = os.path.join("/dev/shm", name.lstrip("/"))
    try:
        with open(path, "rb") as f:
            text = f.read().split(b"\0", 1)[0].decode(errors="replace")
    except OSError:
        return None
    m = _SEQ.search(text)
    seq = int(m.group(1)) if m else 0
    return seq, {k: float(v) for k, v in _P.findall(text)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("name")
    ap.add_argument("--interval", type=float, default=0.5)
    ap.add_argument("--count", type=int, default=0, help="refreshes before exiting (0 = until the segment disappears)")
    a = ap.parse_args(argv)
    prev = {}
    n = 0
    while True:
        snap = read(a.name)
        if snap is None:
            print(f"no segment /dev/shm/{a.name.lstrip('/')}", file=sys.stderr)
            return 1
        seq, vals = snap
        print(f"--- {a.name} seq {seq}")
        for k in sorted(vals):
            d = vals[k] - prev.get(k, vals[k])
            print(f"{k:40s} {vals[k]:16.6g}  (+{d:.6g})")
        prev = vals
        n += 1
        if a.count and n >= a.count:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
