"""Offline tools for the runtime's binary traces (``<name>-<rank>.prof``,
written when the MCA parameter ``profile_filename`` is set; task events come
from the ``task_profiler`` PINS module, user events from the C API).

    python -m parsec_amd.profiling info   trace-0.prof [trace-1.prof ...]
    python -m parsec_amd.profiling csv    out.csv trace-*.prof
    python -m parsec_amd.profiling chrome out.json trace-*.prof   # chrome://tracing / Perfetto
    python -m parsec_amd.profiling dot-merge out.dot graph-*.dot

File layout (profiling.cpp: profiling_dump): magic ``PAMDPRF2``; u32 rank,
n_dict, n_streams, n_infos; u64 t0; infos (key, value strings); dictionary
entries (name, attributes, info description, u64 info length); per stream:
name, i32 thread id, u32 n_infos + that many (key, value) strings, u64 n_events, events (32 B each: u16 key, u16 flags,
u32 taskpool id, u64 event id, u64 timestamp ns, u32 info offset, u32 info
length), u64 info blob size + blob. Strings are u32 length + bytes.

Parity: reference tools/profiling/dbpreader.c (reader), dbpinfos (summary),
python/pbt2ptt.pyx + profile2h5.py (table conversion), h5totrace.py (trace
viewer export), parsec-dotmerger (DOT merge).
"""
import json
import re
import struct
import sys

import numpy as np

EVENT_DTYPE = np.dtype([("key", "<u2"), ("flags", "<u2"), ("taskpool_id", "<u4"), ("event_id", "<u8"),
                        ("timestamp", "<u8"), ("info_off", "<u4"), ("info_len", "<u4")])
assert EVENT_DTYPE.itemsize == 32

_CTYPES = {"int8_t": "b", "uint8_t": "B", "int16_t": "h", "uint16_t": "H", "int32_t": "i", "uint32_t": "I", "int": "i",
           "int64_t": "q", "uint64_t": "Q", "double": "d", "float": "f"}


class Trace:
    def __init__(self, rank, t0, infos, dictionary, streams):
        self.rank = rank
        self.t0 = t0
        self.infos = infos
        self.dictionary = dictionary  # list of dicts: name, attributes, info_desc, info_length
        self.streams = streams        # list of dicts: name, thread_id, events (structured array), info (bytes)


def _rstr(buf, off):
    (n,) = struct.unpack_from("<I", buf, off)
    off += 4
    return buf[off:off + n].decode("utf-8", "replace"), off + n


def read_trace(path):
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:8] not in (b"PAMDPRF1", b"PAMDPRF2"):
        raise ValueError(f"{path}: not a parsec-amd trace")
    v2 = buf[:8] == b"PAMDPRF2"  # per-stream key / value infos
    rank, ndict, nstreams, ninfos = struct.unpack_from("<4I", buf, 8)
    (t0,) = struct.unpack_from("<Q", buf, 24)
    off = 32
    infos = {}
    for _ in range(ninfos):
        k, off = _rstr(buf, off)
        v, off = _rstr(buf, off)
        infos[k] = v
    dictionary = []
    for _ in range(ndict):
        name, off = _rstr(buf, off)
        attr, off = _rstr(buf, off)
        desc, off = _rstr(buf, off)
        (il,) = struct.unpack_from("<Q", buf, off)
        off += 8
        dictionary.append({"name": name, "attributes": attr, "info_desc": desc, "info_length": il})
    streams = []
    for _ in range(nstreams):
        name, off = _rstr(buf, off)
        (tid,) = struct.unpack_from("<i", buf, off)
        off += 4
        sinfos = {}
        if v2:
            (ni,) = struct.unpack_from("<I", buf, off)
            off += 4
            for _ in range(ni):
                k, off = _rstr(buf, off)
                v, off = _rstr(buf, off)
                sinfos[k] = v
        (n,) = struct.unpack_from("<Q", buf, off)
        off += 8
        ev = np.frombuffer(buf, dtype=EVENT_DTYPE, count=n, offset=off).copy()
        off += n * EVENT_DTYPE.itemsize
        (isz,) = struct.unpack_from("<Q", buf, off)
        off += 8
        info = buf[off:off + isz]
        off += isz
        streams.append({"name": name, "thread_id": tid, "events": ev, "info": info, "infos": sinfos})
    return Trace(rank, t0, infos, dictionary, streams)


def _info_fields(desc):
    """'size{int64_t};key{uint64_t};locals{int32_t[2]}' -> [(name, fmt, count)]"""
    out = []
    for part in filter(None, desc.split(";")):
        m = re.match(r"\s*(\w+)\{(\w+)(?:\[(\d+)\])?\}", part)
        if m and m.group(2) in _CTYPES:
            out.append((m.group(1), _CTYPES[m.group(2)], int(m.group(3) or 1)))
    return out


def _decode_info(fields, blob):
    """Fields laid out as the C struct the convertor describes: each at its
    natural alignment (an int32_t followed by a double starts the double at 8)."""
    vals, off = {}, 0
    for name, fmt, cnt in fields:
        align = struct.calcsize("<" + fmt)
        off = (off + align - 1) // align * align
        sz = struct.calcsize("<" + fmt * cnt)
        if off + sz > len(blob):
            break
        v = struct.unpack_from("<" + fmt * cnt, blob, off)
        vals[name] = v[0] if cnt == 1 else list(v)
        off += sz
    return vals


def intervals(traces):
    """Match begin (even key) / end (odd key) events into rows: within each
    stream first, then the begins and ends left over are matched across the
    streams of a rank (an event a task begins on one thread and ends on
    another, e.g. a body that returned ASYNC and ran again elsewhere;
    reference dbpreader.c matches across threads the same way)."""
    rows = []
    for tr in traces:
        fields = [_info_fields(d["info_desc"]) for d in tr.dictionary]

        def row(sb, b, se, e):
            d = int(e["key"]) // 2
            r = {"rank": tr.rank, "stream": sb["name"], "thread": sb["thread_id"],
                 "type": tr.dictionary[d]["name"] if d < len(tr.dictionary) else str(d),
                 "taskpool_id": int(e["taskpool_id"]), "event_id": int(e["event_id"]),
                 "begin": int(b["timestamp"]), "end": int(e["timestamp"]),
                 "duration": int(e["timestamp"]) - int(b["timestamp"])}
            if se is not sb:
                r["end_stream"] = se["name"]
            for st, src in ((sb, b), (se, e)):
                if src["flags"] & 1 and d < len(fields):
                    blob = st["info"][int(src["info_off"]):int(src["info_off"]) + int(src["info_len"])]
                    r.update(_decode_info(fields[d], blob))
            return r

        left_b, left_e = {}, []
        for s in tr.streams:
            open_ = {}
            for e in s["events"]:
                k = int(e["key"])
                ident = (k // 2, int(e["taskpool_id"]), int(e["event_id"]))
                if k % 2 == 0:
                    if ident in open_:  # an earlier begin of this id never ended here
                        left_b.setdefault(ident, []).append((s, open_[ident]))
                    open_[ident] = e
                    continue
                b = open_.pop(ident, None)
                if b is None:
                    left_e.append((ident, s, e))
                    continue
                rows.append(row(s, b, s, e))
            for ident, b in open_.items():
                left_b.setdefault(ident, []).append((s, b))
        for lst in left_b.values():
            lst.sort(key=lambda x: int(x[1]["timestamp"]))
        left_e.sort(key=lambda x: int(x[2]["timestamp"]))
        for ident, se, e in left_e:
            cands = left_b.get(ident)
            if not cands:
                continue
            # the latest begin before this end
            i = max((j for j, (_, b) in enumerate(cands) if int(b["timestamp"]) <= int(e["timestamp"])), default=None)
            if i is None:
                continue
            sb, b = cands.pop(i)
            rows.append(row(sb, b, se, e))
    return rows


def to_dataframe(traces):
    import pandas as pd

    return pd.DataFrame(intervals(traces))


def summary(traces):
    stats = {}
    for r in intervals(traces):
        s = stats.setdefault(r["type"], [0, 0, None, None])
        s[0] += 1
        s[1] += r["duration"]
        s[2] = r["begin"] if s[2] is None else min(s[2], r["begin"])
        s[3] = r["end"] if s[3] is None else max(s[3], r["end"])
    return {k: {"count": v[0], "total_ns": v[1], "avg_ns": v[1] / max(v[0], 1), "first_ns": v[2], "last_ns": v[3]} for k, v in stats.items()}


def to_chrome(traces, path):
    events = [{"name": r["type"], "ph": "X", "ts": r["begin"] / 1e3, "dur": r["duration"] / 1e3, "pid": r["rank"],
               "tid": r["stream"], "args": {k: v for k, v in r.items() if k not in ("rank", "stream", "type", "begin", "end", "duration")}}
              for r in intervals(traces)]
    with open(path, "w") as f:
        json.dump({"traceEvents": events, "displayTimeUnit": "ns"}, f)


def dot_merge(paths, out):
    """Merge the per-rank DOT files written by the grapher (``--dot``)."""
    nodes, edges = [], []
    for p in paths:
        with open(p) as f:
            for line in f:
                line = line.strip()
                if not line or line.startswith("digraph") or line == "}":
                    continue
                (edges if "->" in line else nodes).append(line)
    with open(out, "w") as f:
        f.write("digraph G {\n")
        for l in nodes + edges:
            f.write("  " + l + "\n")
        f.write("}\n")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 1
    cmd = argv.pop(0)
    if cmd == "info":
        trs = [read_trace(p) for p in argv]
        for tr in trs:
            print(f"rank {tr.rank}: {len(tr.streams)} streams, {sum(len(s['events']) for s in tr.streams)} events, infos {tr.infos}")
        for name, s in sorted(summary(trs).items()):
            print(f"  {name:32s} count {s['count']:8d}  total {s['total_ns'] / 1e6:10.3f} ms  avg {s['avg_ns'] / 1e3:10.3f} us")
    elif cmd == "csv":
        to_dataframe([read_trace(p) for p in argv[1:]]).to_csv(argv[0], index=False)
    elif cmd == "chrome":
        to_chrome([read_trace(p) for p in argv[1:]], argv[0])
    elif cmd == "dot-merge":
        dot_merge(argv[1:], argv[0])
    else:
        print(f"unknown command {cmd}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
