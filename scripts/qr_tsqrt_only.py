"""TSQRT (512 + 512) x 512 and GEQRT 512 x 512 panels only, for PMC passes."""
import sys
import torch
sys.path.insert(0, "/root/repo")
import parsec_amd as pa  # noqa: E402
pa.require_native()
nb = 512
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(0)
A1 = torch.triu(torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g))
A2 = torch.rand((nb, nb), dtype=torch.float64, device=dev, generator=g)
T = torch.zeros((nb, nb), dtype=torch.float64, device=dev)
for _ in range(4):
    pa._C.kernel_qr_panel(A1.data_ptr(), nb, A2.data_ptr(), nb, T.data_ptr(), nb, 0, nb, nb, nb, s)
torch.cuda.synchronize()
print("ok")
import os
if os.environ.get("PARSEC_QR_PROFILE"):
    names = ["step1", "barA", "sqrtdiv", "tcol", "dot", "barB", "update", "-"]
    v = pa._C.kernel_qr_profile()
    if v:
        for w in range(4):
            tot = sum(v[w * 8:(w + 1) * 8])
            print(f"wave {w}: " + " ".join(f"{n}={v[w*8+i]/tot:.1%}" for i, n in enumerate(names)) + f"  total={tot/4/16/32:.0f} cyc/col")
