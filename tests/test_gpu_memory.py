"""GPU tile cache under memory pressure and data_advise (reference:
transfer_gpu.c:221-337 W2R write-back task, device_cuda_module.c:1612-1679
prefetch / preferred-device advice, tests/dsl/ptg/cuda/stress.jdf memory
pressure): DPOTRF on host-resident tiles with the cache capped well below the
matrix, checked against the matrix it factors."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp", "gpu_evict.py")


def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("N,nb,frac,prefetch", [(4096, 512, 0.25, 0), (4096, 256, 0.3, 1), (4096, 512, 2.0, 1), (16384, 1024, 0.25, 0)])
def test_dpotrf_forced_eviction(pa, N, nb, frac, prefetch):
    _gpu()
    r = subprocess.run([sys.executable, WORKER, str(N), str(nb), str(frac), str(prefetch)], capture_output=True, text=True, timeout=150)
    print(r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-2000:])
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]


TWO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp", "gpu_two_devices.py")


@pytest.mark.parametrize("N,nb,frac", [(4096, 512, 0.0), (4096, 256, 0.3)])
def test_dpotrf_two_logical_devices(pa, N, nb, frac):
    """DPOTRF on host tiles with the GPU registered as two devices
    (device_hip_replicas 2): both devices run tasks, tiles move between them
    device to device (newest version on the other device, or a read-only input
    staged from the other device's copy), with and without a capped tile cache."""
    _gpu()
    r = subprocess.run([sys.executable, TWO, str(N), str(nb), str(frac)], capture_output=True, text=True, timeout=150)
    print(r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-2000:])
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
