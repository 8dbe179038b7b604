"""Diagnostic: repeat the tile POTRF (+ W = L^-1) kernel sequence and check every
result, optionally while another process keeps the GPU busy with GEMMs.
usage: stress_potrf_tile.py potrf|load N_ITERS [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import parsec_amd as pa  # noqa: E402


def main():
    mode, iters = sys.argv[1], int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    if mode == "load":
        N = 1024
        A = [torch.randn(N, N, dtype=torch.float64, device=dev) for _ in range(8)]
        C = [torch.randn(N, N, dtype=torch.float64, device=dev) for _ in range(8)]
        d = [(a.data_ptr(), a.data_ptr(), c.data_ptr(), N, N, N, N, N, N, -1.0, 1.0, 1, 0) for a, c in zip(A, C)]
        t0 = time.time()
        k = 0
        while time.time() - t0 < iters:
            pa.kernel_dgemm_batch(d, s)
            k += 1
            if k % 50 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print(f"load done {k} launches")
        return
    g = torch.Generator(device=dev).manual_seed(1)
    bad = 0
    for it in range(iters):
        R = torch.randn((n, n), dtype=torch.float64, device=dev, generator=g)
        S = R @ R.t() / n + torch.eye(n, dtype=torch.float64, device=dev)
        A = S.t().contiguous().t().clone()
        W = torch.full((n, n), 7.0, dtype=torch.float64, device=dev).t()
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        if mode == "potrf":
            pa.kernel_dpotrf_w(A.data_ptr(), n, n, info.data_ptr(), W.data_ptr(), n, s)
        else:
            pa.kernel_dpotrf(A.data_ptr(), n, n, info.data_ptr(), s)
        torch.cuda.synchronize()
        L = torch.tril(A)
        r = ((L @ L.t() - S).norm() / S.norm()).item()
        w = (W @ L - torch.eye(n, dtype=torch.float64, device=dev)).abs().max().item() if mode == "potrf" else 0.0
        if r > 1e-13 or w > 1e-10 or info.item() != 0:
            bad += 1
            if bad <= 5:
                E = (L @ L.t() - S).abs()
                rows = (E.max(dim=1).values > 1e-10).nonzero().flatten().tolist()
                print(f"iter {it}: residual {r:.2e} winv {w:.2e} info {info.item()} bad rows {rows[:8]}..{rows[-3:] if rows else ''}", flush=True)
    print(f"{mode} n={n}: {bad}/{iters} bad", flush=True)


if __name__ == "__main__":
    main()
