"""PTG Cholesky (the ptgpp-compiled dpotrf_L.jdf taskpool) through the GPU engine
(HBM-resident and host-resident tiles)."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _spd(N, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    R = torch.rand((N, N), dtype=torch.float64, device=dev, generator=g)
    return (R + R.t()) / 2 + N * torch.eye(N, dtype=torch.float64, device=dev)


@pytest.mark.parametrize("fuse,inplace", [(0, 0), (1, 0), (0, 1)])
@pytest.mark.parametrize("N,nb", [(1024, 256), (2048, 512), (1536, 384)])
def test_dpotrf_hbm_resident(pa, N, nb, fuse, inplace):
    """fuse = 1: POTRF(k) applies SYRK(k-1,k) itself (pre-GEMM in its launch on
    the critical stream); inplace = 1: the panel-solve W-GEMM runs in place
    (ordered row-block signalling, no B-tile copies). The factor is checked
    against torch's fp64 Cholesky."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = pa.init(3)
    prev = pa.dpotrf_fuse_syrk(fuse)
    prev_ip = pa.trsm_inplace(inplace)
    try:
        gpu = pa.first_gpu_device_index()
        NT = N // nb
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        S = _spd(N, "cuda")
        store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        torch.cuda.synchronize()
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        assert pa.read_int(info) == 0
        L = torch.tril(store.permute(1, 3, 0, 2).reshape(N, N))
        assert (torch.linalg.norm(L @ L.t() - S) / torch.linalg.norm(S)).item() < 1e-13
        Lref = torch.linalg.cholesky(S)
        assert (torch.linalg.norm(L - Lref) / torch.linalg.norm(Lref)).item() < 1e-12
        gpus = [d for d in pa.devices() if d["type"] == pa.DEV_HIP]
        assert gpus and gpus[0]["executed_tasks"] > 0
    finally:
        pa.dpotrf_fuse_syrk(prev)
        pa.trsm_inplace(prev_ip)
        ctx.fini()


@pytest.mark.parametrize("sort_pending", [1, 2])
def test_dpotrf_host_resident_staged(pa, sort_pending):
    """Tiles live on the host: the engine stages them into its HBM tile cache
    and pushes final tiles back (collection write-back). sort_pending 2: the
    pending GPU tasks whose data is already on the device go first (reference
    parsec_gpu_sort_pending_list), priority among equals."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np

    N, nb = 1024, 256
    pa.mca_set("device_hip_sort_pending_tasks", str(sort_pending))
    ctx = pa.init(3)
    try:
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N)
        S = _spd(N, "cpu", 3).numpy()
        for m in range(A.mt):
            for n in range(A.nt):
                A.tile(m, n)[:, :] = S[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb]
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        L = np.zeros((N, N))
        for m in range(A.mt):
            for n in range(m + 1):
                L[m * nb:(m + 1) * nb, n * nb:(n + 1) * nb] = A.tile(m, n)
        L = np.tril(L)
        assert np.linalg.norm(L @ L.T - S) / np.linalg.norm(S) < 1e-13
        gpus = [d for d in pa.devices() if d["type"] == pa.DEV_HIP]
        assert gpus[0]["bytes_in"] > 0
    finally:
        ctx.fini()
        pa.mca_set("device_hip_sort_pending_tasks", "1")


def _gpu_matrix(pa, gpu, M, N, mb, nb, fill):
    MT, NT = -(-M // mb), -(-N // nb)
    store = torch.full((NT, MT, nb, mb), float(fill), dtype=torch.float64, device="cuda")
    A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, mb, nb, M, N, device=gpu, ptr=store.data_ptr())
    return A, store


def _dense_of(store, M, N, mb, nb):
    """A dense COPY of the tiled store (the permuted reshape cannot be a view)."""
    NT, MT = store.shape[0], store.shape[1]
    return store.permute(1, 3, 0, 2).reshape(MT * mb, NT * nb)[:M, :N]


def _fill_store(store, dense, mb, nb):
    NT, MT = store.shape[0], store.shape[1]
    pad = torch.zeros((MT * mb, NT * nb), dtype=store.dtype, device=store.device)
    pad[:dense.shape[0], :dense.shape[1]] = dense
    store.copy_(pad.reshape(MT, mb, NT, nb).permute(2, 0, 3, 1))


@pytest.mark.parametrize("smb,dmb,win", [(64, 40, (150, 130, 7, 33, 21, 2)), (64, 64, (128, 192, 64, 0, 0, 128))])
def test_redistribute_hbm_resident(pa, smb, dmb, win):
    """redistribute.jdf / redistribute_reshuffle.jdf on matrices living in HBM:
    the HIP bodies (strided device copies) run, nothing is staged to the host."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        S, s_store = _gpu_matrix(pa, gpu, 300, 260, smb, smb, 0.0)
        T, t_store = _gpu_matrix(pa, gpu, 280, 320, dmb, dmb, -1.0)
        src = torch.arange(300 * 260, dtype=torch.float64, device="cuda").reshape(300, 260)
        _fill_store(s_store, src, smb, smb)
        torch.cuda.synchronize()
        before = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]
        sr, sc, si, sj, ti, tj = win
        assert pa.redistribute(ctx, S, T, sr, sc, si, sj, ti, tj) == 0
        torch.cuda.synchronize()
        after = [d for d in pa.devices() if d["type"] == pa.DEV_HIP][0]
        want = torch.full((280, 320), -1.0, dtype=torch.float64, device="cuda")
        want[ti:ti + sr, tj:tj + sc] = src[si:si + sr, sj:sj + sc]
        assert torch.equal(_dense_of(t_store, 280, 320, dmb, dmb), want)
        assert after["executed_tasks"] > before["executed_tasks"]
        assert after["bytes_in"] == before["bytes_in"]  # device to device only
    finally:
        ctx.fini()


def _factor_gpu(pa, S, N, nb, mode, limit=0.0):
    """JDF Cholesky of S (torch, cuda) in panel-solve mode `mode`; returns L."""
    prev_limit = pa.trsm_inverse_limit()
    prev = pa.trsm_inverse_mode(mode, limit)
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        NT = N // nb
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        torch.cuda.synchronize()
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        assert pa.read_int(info) == 0
        return torch.tril(store.permute(1, 3, 0, 2).reshape(N, N)).clone()
    finally:
        ctx.fini()
        pa.trsm_inverse_mode(prev, prev_limit)


@pytest.mark.parametrize("nb", [128, 256, 512, 1024])
def test_trsm_inverse_modes_gpu(pa, nb):
    """Panel solve through W = L^-1 (mode 0), by substitution (mode 2) and auto
    (mode 1). Auto decides per panel from max|L| max|W|: by default the tile
    POTRF publishes it to pinned host memory and the TRSM launch picks the
    route on the host (no gated kernel); with trsm_estimate_route(0) the copy
    kernel estimates into workspace slots, the W-GEMM skips and the in-place
    gated substitution kernel solves above the limit. The panel tile is the
    packed one POTRF sends (W below, L(k,k)^T above the diagonal): the W-GEMM
    reads W unpacked in the workspace, the substitution reads L from the tile.
    On an SPD matrix with cond 1e12 (numerics sweep:
    profiles/r4_trsm_inverse_numerics.txt) every mode is backward stable; auto
    with its default limit takes the inverse path (same factor as mode 0) and
    auto with limit 1 takes the substitution path (same factor as mode 2),
    through either estimate route, at every tile size."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N = 2048
    g = torch.Generator(device="cpu").manual_seed(11)
    q, _ = torch.linalg.qr(torch.randn((N, N), dtype=torch.float64, generator=g))
    S = ((q * torch.logspace(0, -12, N, dtype=torch.float64)) @ q.t())
    S = (0.5 * (S + S.t())).cuda()
    L0 = _factor_gpu(pa, S, N, nb, 0)
    L2 = _factor_gpu(pa, S, N, nb, 2)
    pa.trsm_estimate_stats(True)
    L1 = _factor_gpu(pa, S, N, nb, 1)
    L1s = _factor_gpu(pa, S, N, nb, 1, 1.0)
    published, host, device = pa.trsm_estimate_stats(True)
    NT = N // nb
    assert published == 2 * (NT - 1)           # every POTRF with a W published its estimate
    assert host == 2 * NT * (NT - 1) // 2      # every TRSM decided on the host
    assert device == 0
    prev_route = pa.trsm_estimate_route(0)
    try:
        L1d = _factor_gpu(pa, S, N, nb, 1)
        L1ds = _factor_gpu(pa, S, N, nb, 1, 1.0)
    finally:
        pa.trsm_estimate_route(prev_route)
    published, host, device = pa.trsm_estimate_stats(True)
    assert published == 0 and host == 0
    assert device == 2 * NT * (NT - 1) // 2
    nS = torch.linalg.norm(S)
    for L in (L0, L1, L2, L1s, L1d, L1ds):
        assert (torch.linalg.norm(L @ L.t() - S) / nS).item() < 1e-14
    d02 = torch.linalg.norm(L0 - L2).item()
    assert d02 > 0  # the two solves differ (by ~cond(L(k,k)) eps)
    for La, Lb in ((L1, L0), (L1d, L0)):  # auto below the limit = the inverse path
        assert torch.linalg.norm(La - Lb).item() < 1e-3 * d02
    for La, Lb in ((L1s, L2), (L1ds, L2)):  # auto above it = the substitution path
        assert torch.linalg.norm(La - Lb).item() < 1e-3 * d02


def test_trsm_estimate_forgotten_on_reuse(pa):
    """A panel estimate is keyed by the address of the W its POTRF wrote. Once
    that W is gone, a buffer carved at the same address (a receive buffer, a
    re-staged tile) is a different tile: the lookup must not return the old
    estimate (it would skip the guard of an ill-conditioned panel that arrived
    from another rank). Every tile-cache allocation drops the key of its
    address. Here the first context's zone (and its W tiles) is released at
    fini; the next context's zone is carved from the same device memory."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N, nb = 2048, 256
    NT = N // nb
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        S = _spd(N, "cuda", 7)
        store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
        torch.cuda.synchronize()
        tp, info = pa.dpotrf_jdf_new(A)
        ctx.add_taskpool(tp)
        ctx.start()
        ctx.wait()
        assert pa.read_int(info) == 0
        known = set(pa.trsm_estimate_known())
        assert len(known) >= NT - 1, known
        assert all(pa.trsm_estimate_lookup(p) > 0 for p in known)
    finally:
        ctx.fini()
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        got, hits = [], []
        for _ in range(4 * NT):
            p = pa.device_cache_alloc(gpu, nb * nb * 8)
            if not p:
                break
            got.append(p)
            if p in known:
                hits.append(p)
        for p in got:
            pa.device_cache_free(gpu, p)
        if not hits:
            pytest.skip("the new zone did not reuse a W address")
        assert all(pa.trsm_estimate_lookup(p) == 0.0 for p in hits)
        assert all(pa.trsm_estimate_lookup(p) > 0 for p in known - set(hits))  # only the reused keys went
    finally:
        ctx.fini()


@pytest.mark.parametrize("hp_route", [1, 2])
@pytest.mark.parametrize("N,nb", [(4096, 256), (4096, 512)])
def test_dpotrf_early_release(pa, N, nb, hp_route):
    """device_hip_early_release=1: critical-stream groups release their tasks'
    successors when launched (the chain POTRF -> TRSM -> SYRK -> POTRF queues
    in stream order; successors on other streams wait for the group's event);
    hp_route 2 puts the non-critical high-priority tasks on their own stream.
    The factor matches and tasks were released early."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    pa.mca_set("device_hip_early_release", "1")
    pa.mca_set("device_hip_hp_on_critical_stream", str(hp_route))
    ctx = pa.init(3)
    try:
        gpu = pa.first_gpu_device_index()
        NT = N // nb
        store = torch.empty((NT, NT, nb, nb), dtype=torch.float64, device="cuda")
        A = pa.BlockCyclic(pa.MATRIX_DOUBLE, 0, nb, nb, N, N, device=gpu, ptr=store.data_ptr())
        S = _spd(N, "cuda", 5)
        for rep in range(2):
            store.copy_(S.reshape(NT, nb, NT, nb).permute(2, 0, 3, 1))
            torch.cuda.synchronize()
            tp, info = pa.dpotrf_jdf_new(A)
            ctx.add_taskpool(tp)
            ctx.start()
            ctx.wait()
            assert pa.read_int(info) == 0
            torch.cuda.synchronize()
            L = torch.tril(store.permute(1, 3, 0, 2).reshape(N, N))
            assert (torch.linalg.norm(L @ L.t() - S) / torch.linalg.norm(S)).item() < 1e-13, rep
        gpus = [d for d in pa.devices() if d["type"] == pa.DEV_HIP]
        assert gpus[0]["early_released"] >= 2 * NT, gpus[0]
    finally:
        ctx.fini()
        pa.mca_set("device_hip_early_release", "0")
        pa.mca_set("device_hip_hp_on_critical_stream", "1")
