"""One grouped GEMM workload for counter collection: 40 tasks of 1024^3 (C -= A B^T), 20 launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parsec_amd as pa  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
nb, ntask = 1024, 40
A = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(8)]
C = [torch.randn(nb, nb, dtype=torch.float64, device=dev) for _ in range(ntask)]
descs = [(A[i % 8].data_ptr(), A[(i + 1) % 8].data_ptr(), C[i].data_ptr(), nb, nb, nb, nb, nb, nb, -1.0, 1.0, 1, 0) for i in range(ntask)]
for _ in range(20):
    pa.kernel_dgemm_batch(descs, s)
torch.cuda.synchronize()
print("done")
