"""Kernel micro-benchmarks on one GPU: grouped fp64 GEMM (our MFMA kernel) vs
torch/rocBLAS, tile TRSM and tile POTRF. Prints one line per measurement."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parsec_amd as pa  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for nb, ntask in ((512, 1), (512, 8), (512, 32), (512, 128), (1024, 1), (1024, 16), (1024, 64)):
        A = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(min(ntask, 8))]
        C = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(ntask)]
        descs = [(A[i % len(A)].data_ptr(), A[(i + 1) % len(A)].data_ptr(), C[i].data_ptr(), nb, nb, nb, nb, nb, nb, -1.0, 1.0, 1, 0) for i in range(ntask)]
        dt = timeit(lambda: pa.kernel_dgemm_batch(descs, s))
        fl = 2.0 * nb ** 3 * ntask
        tt = timeit(lambda: [torch.addmm(C[i], A[i % len(A)], A[(i + 1) % len(A)].t(), beta=1.0, alpha=-1.0, out=C[i]) for i in range(ntask)])
        print(f"gemm nb={nb} tasks={ntask}: ours {fl / dt / 1e12:6.1f} TF ({dt * 1e6:8.1f} us)   torch-loop {fl / tt / 1e12:6.1f} TF", flush=True)
    for n in (4096, 8192):
        A = torch.randn(n, n, dtype=torch.float64, device=dev)
        B = torch.randn(n, n, dtype=torch.float64, device=dev)
        C = torch.zeros(n, n, dtype=torch.float64, device=dev)
        dt = timeit(lambda: pa.kernel_dgemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, 1.0, 0.0, 1, 0, s), 3)
        tt = timeit(lambda: torch.mm(A, B.t(), out=C), 3)
        print(f"gemm n={n}: ours {2 * n ** 3 / dt / 1e12:6.1f} TF   torch {2 * n ** 3 / tt / 1e12:6.1f} TF", flush=True)
    for nb in (512, 1024):
        R = torch.randn(nb, nb, dtype=torch.float64, device=dev)
        S = R @ R.t() + nb * torch.eye(nb, dtype=torch.float64, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        W = S.clone()
        dt = timeit(lambda: (W.copy_(S), pa.kernel_dpotrf(W.data_ptr(), nb, nb, info.data_ptr(), s)))
        L = torch.linalg.cholesky(S)
        B = torch.randn(nb, nb, dtype=torch.float64, device=dev)
        Bw = B.clone()
        tt = timeit(lambda: (Bw.copy_(B), pa.kernel_dtrsm(L.data_ptr(), Bw.data_ptr(), nb, nb, nb, nb, s)))
        print(f"potrf tile nb={nb}: {dt * 1e6:8.1f} us   trsm tile: {tt * 1e6:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
