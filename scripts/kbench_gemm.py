"""Grouped fp64 GEMM throughput for one kernel variant (PARSEC_GEMM_VARIANT /
PARSEC_GEMM_FULL are read once per process): the DPOTRF trailing-update shape
(C -= A B^T on nb x nb tiles) and one large square GEMM."""
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
    tag = f"variant={os.environ.get('PARSEC_GEMM_VARIANT', '0')} full={os.environ.get('PARSEC_GEMM_FULL', '1')}"
    for nb, ntask in ((512, 32), (1024, 16), (1024, 40)):
        A = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(8)]
        C = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(ntask)]
        C0 = [c.clone() for c in C]
        descs = [(A[i % 8].data_ptr(), A[(i + 1) % 8].data_ptr(), C[i].data_ptr(), nb, nb, nb, nb, nb, nb, -1.0, 1.0, 1, 0) for i in range(ntask)]
        pa.kernel_dgemm_batch(descs, s)
        torch.cuda.synchronize()
        err = max(float((C[i] - (C0[i] - A[(i + 1) % 8].t() @ A[i % 8])).abs().max()) for i in range(ntask))  # column-major view
        dt = timeit(lambda: pa.kernel_dgemm_batch(descs, s))
        fl = 2.0 * nb ** 3 * ntask
        print(f"{tag} gemm nb={nb} tasks={ntask}: {fl / dt / 1e12:6.1f} TF ({dt * 1e6:8.1f} us) maxerr={err:.2e}", flush=True)
    n = 8192
    A = torch.randn(n, n, dtype=torch.float64, device=dev)
    B = torch.randn(n, n, dtype=torch.float64, device=dev)
    C = torch.zeros(n, n, dtype=torch.float64, device=dev)
    dt = timeit(lambda: pa.kernel_dgemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, 1.0, 0.0, 1, 0, s), 3)
    print(f"{tag} gemm n={n}: {2 * n ** 3 / dt / 1e12:6.1f} TF", flush=True)


if __name__ == "__main__":
    main()
