"""Grouped tile DGEMM (C -= A B^T, 1024^3 tiles) : this framework's MFMA kernel
vs the vendor library on the same batch (torch.baddbmm -> rocBLAS/hipBLASLt
strided-batched), TFLOP/s for batch sizes the DPOTRF trailing update uses."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parsec_amd as pa  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
nb = 1024


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for ntask in (16, 40, 120, 500):
    A = torch.randn(ntask, nb, nb, dtype=torch.float64, device=dev)
    B = torch.randn(ntask, nb, nb, dtype=torch.float64, device=dev)
    C = torch.randn(ntask, nb, nb, dtype=torch.float64, device=dev)
    C2 = C.clone()
    # column-major tiles: our kernel sees each [nb, nb] row-major tensor as the transposed column-major tile
    descs = [(A[i].data_ptr(), B[i].data_ptr(), C[i].data_ptr(), nb, nb, nb, nb, nb, nb, -1.0, 1.0, 1, 0) for i in range(ntask)]
    flops = 2.0 * nb ** 3 * ntask
    reps = max(2, int(2000 // ntask))
    t_ours = timeit(lambda: pa.kernel_dgemm_batch(descs, s), reps)
    t_vend = timeit(lambda: torch.baddbmm(C2, A, B.transpose(1, 2), beta=1.0, alpha=-1.0, out=C2), reps)
    print(f"ntask {ntask:4d} ours {flops / t_ours / 1e12:6.1f} TF  vendor(baddbmm) {flops / t_vend / 1e12:6.1f} TF", flush=True)
    del A, B, C, C2
    torch.cuda.empty_cache()
