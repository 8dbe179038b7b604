"""Latency of the DPOTRF critical-path kernels on an otherwise idle GPU:
tile POTRF (+W), the panel TRSM of one tile (as GEMM with W, and blocked),
the lower-only SYRK of one tile. Prints microseconds per call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import parsec_amd as pa  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for n in (512, 1024):
        R = torch.randn((n, n), dtype=torch.float64, device=dev)
        S = (R @ R.t() / n + torch.eye(n, dtype=torch.float64, device=dev)).t().contiguous()
        A = S.clone()
        W = torch.empty((n, n), dtype=torch.float64, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        t_pw = timeit(lambda: (A.copy_(S), pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, s)))
        t_p = timeit(lambda: (A.copy_(S), pa.kernel_dpotrf(A.data_ptr(), n, n, info.data_ptr(), s)))
        t_cp = timeit(lambda: A.copy_(S))
        B = torch.randn((n, n), dtype=torch.float64, device=dev)
        t_tw = timeit(lambda: pa.kernel_trsm_w_batch([(B.data_ptr(), W.data_ptr(), n, n, n, n)], s))
        pa.kernel_dpotrf(A.data_ptr(), n, n, info.data_ptr(), s)
        t_tb = timeit(lambda: pa.kernel_dtrsm(A.data_ptr(), B.data_ptr(), n, n, n, n, s))
        C = torch.randn((n, n), dtype=torch.float64, device=dev)
        t_sy = timeit(lambda: pa.kernel_dgemm(B.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, 1, s))
        t_ge = timeit(lambda: pa.kernel_dgemm(B.data_ptr(), A.data_ptr(), C.data_ptr(), n, n, n, n, n, n, -1.0, 1.0, 1, 0, s))
        if os.environ.get("PARSEC_POTRF_STAMPS"):
            A.copy_(S)
            pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, s)
            torch.cuda.synchronize()
            st = pa.kernel_potrf_stamps()
            names = ["start", "enter", "zeroed", "p0 panel", "p0 rest", "p1 panel", "p1 rest", "p2 panel", "p2 rest", "p3 panel", "p3 rest", "row3 inv", "-", "end"]
            print(f"n={n} last DIAG phases (us): " + " ".join(f"{names[i]} {(st[i] - st[i - 1]) / 100:.2f}" for i in range(1, 14)), flush=True)
        prev = pa.kernel_potrf_steps(0)
        t_pw0 = timeit(lambda: (A.copy_(S), pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, s)))
        t_p0 = timeit(lambda: (A.copy_(S), pa.kernel_dpotrf(A.data_ptr(), n, n, info.data_ptr(), s)))
        pa.kernel_potrf_steps(prev)
        print(f"n={n}: 3-launch path: potrf+W {t_pw0 - t_cp:.1f} us, potrf {t_p0 - t_cp:.1f} us", flush=True)
        print(f"n={n}: potrf+W {t_pw - t_cp:.1f} us, potrf {t_p - t_cp:.1f} us, trsm-as-gemm {t_tw:.1f} us, trsm-blocked {t_tb:.1f} us, "
              f"syrk {t_sy:.1f} us, gemm {t_ge:.1f} us (copy {t_cp:.1f})", flush=True)


if __name__ == "__main__":
    main()
