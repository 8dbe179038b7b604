"""Practical HBM bandwidth of one MI355X for a streaming kernel: torch device
copy (read + write) of large fp64 buffers and a read-mostly reduction."""
import time

import torch

dev = torch.device("cuda", 0)
for gib in (1, 4):
    n = gib * (1 << 30) // 8
    a = torch.rand(n, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 10
    for _ in range(reps):
        b.copy_(a)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(f"copy {gib} GiB: {2 * n * 8 / dt / 1e12:.2f} TB/s (read + write)", flush=True)
    s = a.sum()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        s = a.sum()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(f"sum  {gib} GiB: {n * 8 / dt / 1e12:.2f} TB/s (read)", flush=True)
    del a, b
