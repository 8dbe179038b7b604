"""Phase cycles of the QR sub-panel kernel (qr_sub2c) UNDER LOAD: one DGEQRF of
config 4 (32k / nb 512) with PARSEC_QR_PROFILE=1, then the per-wave phase sums
(v load, column ops, factor + T column, barrier) per sub-panel launch-task,
next to the same numbers for an isolated TSQRT 512 (scripts/qr_sub2_phases.py).
usage: python scripts/qr_phases_loaded.py [N]"""
import os
import sys

os.environ["PARSEC_QR_PROFILE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_workloads as bw  # noqa: E402


class A:
    pass


a = A()
a.n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
a.nb, a.ib, a.steps, a.warmup, a.cores = 512, 32, 1, 0, 4
a.qr_grid, a.share_gpu, a.check, a.qr_tree, a.qr_domain = "2d", False, False, "hqr", 0
out, rank = bw.bench_qr(a)
import parsec_amd as pa  # noqa: E402

v = pa._C.kernel_qr_profile()
ntsqrt = (a.n // a.nb) * (a.n // a.nb - 1) // 2 + a.n // a.nb  # TSQRT + GEQRT panels
names = ["v load", "columns", "factor+T", "barrier"]
print(f"DGEQRF N={a.n}: {out['value']:.0f} GF/s; sub-panel phase cycles per wave, summed over the run; per panel factorization (TSQRT/GEQRT: {ntsqrt})")
for w in range(8):
    row = v[(w & 3) * 8 + (w >> 2) * 4:(w & 3) * 8 + (w >> 2) * 4 + 4]
    tot = sum(row) or 1
    print(f"wave {w}: " + "  ".join(f"{names[i]} {row[i] / ntsqrt / 1e3:8.1f}k ({100 * row[i] / tot:4.1f}%)" for i in range(4)) + f"  total {tot / ntsqrt / 1e3:.1f}k")
