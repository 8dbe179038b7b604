"""GPU-side spans in the trace: every launched kernel group of the HIP device
engine becomes a GPU_EXEC begin/end pair measured with HIP timing events and
converted to the profiling clock (reference device_cuda_module.c:1427-1469 and
2306-2329 record exec / movein / moveout events on the device streams)."""
import pytest

from parsec_amd import profiling

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_gpu_exec_spans(pa, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    base = str(tmp_path / "gtrace")
    pa.mca_set("profile_filename", base)
    pa.mca_set("mca_pins", "task_profiler")
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("profile_filename")
        pa.mca_unset("mca_pins")
    N, nb = 4096, 512
    NT = N // nb
    g = torch.Generator(device="cuda").manual_seed(3)
    R = torch.randn((N, N), dtype=torch.float64, device="cuda", generator=g)
    S = R @ R.t() / N + torch.eye(N, dtype=torch.float64, device="cuda")
    store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
    store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=pa.first_gpu_device_index(), ptr=store.data_ptr())
    torch.cuda.synchronize()
    tp, info = pa.dpotrf_jdf_new(A)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    assert pa.read_int(info) == 0
    ctx.fini()
    tr = profiling.read_trace(base + "-0.prof")
    rows = [r for r in profiling.intervals([tr]) if r["type"] == "GPU_EXEC"]
    assert rows, "no GPU spans in the trace"
    assert all(r["duration"] > 0 for r in rows)
    assert sum(r["ntasks"] for r in rows) >= NT * (NT + 1) * (NT + 2) // 6
    # one HIP stream executes its groups in order: spans of a stream never overlap
    by = {}
    for r in rows:
        by.setdefault(r["stream"], []).append((r["begin"], r["end"]))
    for spans in by.values():
        spans.sort()
        assert all(a[1] <= b[0] + 2000 for a, b in zip(spans, spans[1:]))  # 2 us clock slack


def test_gpu_copy_spans(pa, tmp_path):
    """Host-resident tiles: every stage-in is a GPU_MOVEIN span and every
    write-back a GPU_MOVEOUT span on the device's copy stream, timed by HIP
    events (reference device_cuda_module.c:1442-1453, 2317-2321 movein /
    moveout events), with the bytes moved."""
    import numpy as np

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    base = str(tmp_path / "ctrace")
    pa.mca_set("profile_filename", base)
    try:
        ctx = pa.init(2)
    finally:
        pa.mca_unset("profile_filename")
    N, nb = 1024, 256
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
    rng = np.random.default_rng(5)
    R = rng.random((N, N))
    S = R @ R.T / N + np.eye(N)
    for m in range(A.mt):
        for n in range(A.nt):
            A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
    tp, info = pa.dpotrf_jdf_new(A)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    assert pa.read_int(info) == 0
    ctx.fini()
    tr = profiling.read_trace(base + "-0.prof")
    rows = profiling.intervals([tr])
    movein = [r for r in rows if r["type"] == "GPU_MOVEIN"]
    moveout = [r for r in rows if r["type"] == "GPU_MOVEOUT"]
    NT = N // nb
    assert len(movein) >= NT * (NT + 1) // 2  # every lower tile came in at least once
    assert len(moveout) >= NT * (NT + 1) // 2  # and went home
    assert all(r["bytes"] == nb * nb * 8 and r["duration"] >= 0 for r in movein + moveout)
