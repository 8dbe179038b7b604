"""parsec-amd: a task-DAG runtime for AMD MI355X (gfx950) nodes.

PaRSEC-style Parameterized Task Graphs (PTG, `.jdf` compiled by `ptgpp`) and
Dynamic Task Discovery (DTD) over a native C++/HIP runtime: work-stealing
priority schedulers, a GPU engine with one manager thread per GPU, batched
CDNA4 MFMA tile kernels, shared-memory active messages + RCCL data plane
between ranks, termination detection and tracing.

Import order matters on ROCm: torch (if installed) is imported first so the
native library binds to the same HIP runtime instance as PyTorch.
"""
import os as _os

ROOT = _os.path.dirname(_os.path.abspath(__file__))
LIB = _os.path.join(ROOT, "lib", "libparsec_amd.so")

try:  # bind to torch's HIP runtime when torch is present
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover
    _torch = None

try:
    from . import _C  # noqa: E402
    from ._C import *  # noqa: F401,F403,E402
    from .runtime import init, Context, dtd_taskpool, insert_task  # noqa: E402,F401
    NATIVE_ERROR = None
except ImportError as _e:  # native extension not built yet (python -m parsec_amd._build)
    _C = None
    NATIVE_ERROR = _e


def native_available():
    return _C is not None


def require_native():
    if _C is None:
        raise ImportError(f"parsec_amd native extension missing: {NATIVE_ERROR}; run `python -m parsec_amd._build`")
    return _C
