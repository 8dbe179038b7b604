"""Pythonic helpers over the native runtime (parsec_amd._C)."""
from . import _C

Context = _C.Context


def init(nb_cores=-1, args=None, **mca):
    """Create a runtime context (reference: parsec_init).

    Keyword arguments are MCA parameters, e.g. ``init(4, sched="lfq")`` is the
    same as ``--mca mca_sched lfq``; names are given without the ``mca_`` prefix
    only for the selector params (sched, pins).
    """
    for k, v in mca.items():
        name = {"sched": "mca_sched", "pins": "mca_pins"}.get(k, k)
        _C.mca_set(name, str(v))
    return _C.Context(nb_cores, list(args or []))


def dtd_taskpool(ctx=None):
    tp = _C.DtdTaskpool()
    if ctx is not None:
        ctx.add_taskpool(tp)
    return tp


_class_cache = {}


def _param_of(arg):
    obj, op = arg[0], arg[1]
    kind = op & 0xF00000
    if kind == _C.VALUE:
        if isinstance(obj, float):
            return (op, 8)
        if isinstance(obj, bytes):
            return (op, len(obj))
        return (op, arg[2] if len(arg) > 2 else 4)
    if kind == _C.SCRATCH:
        return (op, int(obj))
    return (op, _C.PASSED_BY_REF)


def insert_task(tp, fn, args, priority=0, name=None, gpu=None):
    """Insert a DTD task (reference: parsec_dtd_insert_task).

    ``fn(task)`` is the CPU body (may be None when only a GPU body exists);
    ``gpu`` names a built-in GPU body ("dgemm", "dsyrk", "dtrsm", "dpotrf",
    "memset"). ``args`` is a list of ``(obj, op)`` tuples where obj is a Tile
    for data flows, a python value for VALUE, a size for SCRATCH.
    """
    name = name or getattr(fn, "__name__", None) or (gpu or "task")
    key = (id(tp), name)
    tc = _class_cache.get(key)
    if tc is None:
        tc = tp.task_class(name, [_param_of(a) for a in args])
        if gpu:
            tp.add_chore(tc, _C.DEV_HIP, None, gpu)
        if fn is not None:
            tp.add_chore(tc, _C.DEV_CPU, fn)
        _class_cache[key] = tc
    tp.insert_task(tc, [tuple(a) for a in args], priority)
    return tc
