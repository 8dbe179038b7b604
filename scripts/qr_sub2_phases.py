"""Phase cycles of the QR sub-panel kernel (qr_sub2) for one TSQRT 512 on an idle
MI355X: PARSEC_QR_PROFILE=1 accumulates s_memtime deltas per phase and wave.
Phases (PARSEC_QR_SUB2=0 kernel): 0 sigma+reflector, 1 barrier A, 2 norm/tau, 3 T column, 4 dot, 5 barrier B,
6 update; default column-owner kernel: v load, column ops, factor + T column, barrier."""
import os
import sys

os.environ["PARSEC_QR_PROFILE"] = "1"
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parsec_amd as pa  # noqa: E402

pa.require_native()
_C = pa._C
nb = 512
torch.cuda.set_device(0)
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(0)
A1 = torch.triu(torch.rand((nb, nb), dtype=torch.float64, device="cuda", generator=g))
A2 = torch.rand((nb, nb), dtype=torch.float64, device="cuda", generator=g)
T = torch.zeros((nb, nb), dtype=torch.float64, device="cuda")
_C.kernel_qr_panel(A1.data_ptr(), nb, A2.data_ptr(), nb, T.data_ptr(), nb, 0, nb, nb, nb, s)
torch.cuda.synchronize()
v = _C.kernel_qr_profile()
if os.environ.get("PARSEC_QR_SUB2", "1") == "0":
    names = ["sigma+refl", "barrierA", "norm/tau", "Tcol", "dot", "barrierB", "update", "-"]
    for w in range(4):
        row = v[w * 8:(w + 1) * 8]
        tot = sum(row) or 1
        print(f"wave-slot {w}: " + "  ".join(f"{names[i]} {row[i] / 1e3:9.1f}k ({row[i] / tot:5.1%})" for i in range(7)))
else:  # column-owner kernel: waves w and w+4 of every sub-panel step, 4 phases each
    names = ["v load", "columns", "factor+T", "barrier"]
    for w in range(8):
        row = v[(w & 3) * 8 + (w >> 2) * 4:(w & 3) * 8 + (w >> 2) * 4 + 4]
        tot = sum(row) or 1
        print(f"wave {w}: " + "  ".join(f"{names[i]} {row[i] / 1e3:9.1f}k ({row[i] / tot:5.1%})" for i in range(4)))
