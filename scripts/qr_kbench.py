"""Isolated timing of the QR panel / apply kernels (GEQRT, TSQRT, UNMQR, TSMQR
tile bodies) on one MI355X: wall time per call with the GPU otherwise idle."""
import sys
import time

import torch

sys.path.insert(0, "/root/repo")
import parsec_amd as pa  # noqa: E402

pa.require_native()
_C = pa._C
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(0)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


A1 = torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g)
A2 = torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g)
T = torch.zeros((nb, nb), dtype=torch.float64, device=dev)
V = torch.zeros((nb, nb), dtype=torch.float64, device=dev)
A1b, A2b = A1.clone(), A2.clone()


def geqrt():
    A1.copy_(A1b)
    _C.kernel_qr_panel(A1.data_ptr(), nb, 0, nb, T.data_ptr(), nb, V.data_ptr(), nb, 0, nb, s)


def tsqrt():
    A1.copy_(torch.triu(A1b))
    A2.copy_(A2b)
    _C.kernel_qr_panel(A1.data_ptr(), nb, A2.data_ptr(), nb, T.data_ptr(), nb, 0, nb, nb, nb, s)


C1 = torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g)
C2 = torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g)
ws = torch.empty(2 * nb * nb, dtype=torch.float64, device=dev)


def unmqr():
    _C.kernel_qr_apply(V.data_ptr(), nb, T.data_ptr(), nb, 0, nb, C2.data_ptr(), nb, nb, nb, nb, ws.data_ptr(), s)


def tsmqr():
    _C.kernel_qr_apply(A2.data_ptr(), nb, T.data_ptr(), nb, C1.data_ptr(), nb, C2.data_ptr(), nb, nb, nb, nb, ws.data_ptr(), s)


copy_us = timeit(lambda: (A1.copy_(A1b), A2.copy_(A2b)))
print(f"nb={nb} copies {copy_us:8.1f} us")
for name, fn, fl in (("GEQRT", geqrt, 4 / 3 * nb ** 3), ("TSQRT", tsqrt, 2 * nb ** 3), ("UNMQR", unmqr, 2 * nb ** 3), ("TSMQR", tsmqr, 4 * nb ** 3)):
    us = timeit(fn)
    print(f"nb={nb} {name} {us:9.1f} us  {fl / us / 1e6:7.1f} GF/s", flush=True)
