"""TSMQR-shaped block-reflector applications, batched as the engine launches them
(launch_qr_apply: W = A1 + V^T A2 (TN), W2 = T^T W with A1 -= W2 (TN, lower),
A2 -= V W2 (NN)), nb x nb tiles: rate counted with the executed 5 nb^3 flops and
with the 4 nb^3 the DGEQRF rate uses. Run under rocprofv3 --kernel-trace to split
the three grouped GEMM launches."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parsec_amd as pa  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for nb, cnt in ((512, 32), (512, 64), (1024, 16)):
        V = torch.randn(nb, nb, dtype=torch.float64, device=dev) / nb
        T = torch.tril(torch.randn(nb, nb, dtype=torch.float64, device=dev)) / nb  # column-major view: upper T
        A1 = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(cnt)]
        A2 = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(cnt)]
        ws = torch.empty(pa.kernel_qr_apply_ws(cnt, nb, nb) // 8 + 64, dtype=torch.float64, device=dev)
        ds = [(V.data_ptr(), nb, T.data_ptr(), nb, A1[i].data_ptr(), nb, A2[i].data_ptr(), nb, nb, nb, nb) for i in range(cnt)]
        # reference on the first pair (column-major tiles = transposed torch views)
        a1, a2 = A1[0].t().clone(), A2[0].t().clone()
        v, t = V.t(), T.t()
        W = a1 + v.t() @ a2
        W2 = t.t() @ W
        r1, r2 = a1 - W2, a2 - v @ W2
        pa.kernel_qr_apply_batch(ds[:1], ws.data_ptr(), s)
        torch.cuda.synchronize()
        err = max(float((A1[0].t() - r1).abs().max()), float((A2[0].t() - r2).abs().max()))
        reps = 10
        pa.kernel_qr_apply_batch(ds, ws.data_ptr(), s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            pa.kernel_qr_apply_batch(ds, ws.data_ptr(), s)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"qr_apply nb={nb} x{cnt}: {5 * nb ** 3 * cnt / dt / 1e12:6.1f} TF executed, {4 * nb ** 3 * cnt / dt / 1e12:6.1f} TF counted "
              f"({dt * 1e6:8.1f} us) maxerr={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
