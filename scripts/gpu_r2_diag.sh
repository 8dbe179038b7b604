#!/bin/bash
# 2-rank GPU DGEQRF (1D row-cyclic), repeated, IPC vs host plane
set -o pipefail
mkdir -p gpurun_out/qr
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  rm -f gpurun_out/qr/R*.npy
  for r in 0 1; do env "$@" timeout -k 5 60 python tests/mp/gpu_dist.py dgeqrf $r 2 qr_${name}_$$ 2048 256 2 gpurun_out/qr > gpurun_out/qr_${name}_$r.log 2>&1 & done
  wait
  python - <<'PY'
import numpy as np, torch
R = sum(np.load(f"gpurun_out/qr/R{r}.npy") for r in range(2))
g = torch.Generator().manual_seed(77)
A = (torch.rand((2048, 2048), dtype=torch.float64, generator=g) - 0.5).numpy()
G = A.T @ A
E = np.abs(R.T @ R - G)
bad = sorted({(int(i) // 256, int(j) // 256) for i, j in zip(*np.nonzero(E > 1e-8))})
print(f"rel {np.linalg.norm(R.T @ R - G) / np.linalg.norm(G):.2e} bad blocks {bad[:10]}")
PY
  echo "   ^ $name"
}
for i in 1 2 3; do
run ipc$i A=1
run host$i PARSEC_MCA_comm_device_plane=host
done
