#!/bin/bash
set -o pipefail
bash scripts/gpu/r4_qr_yield.sh || exit 1
bash scripts/gpu/r4_qr_domain.sh || exit 1
ENVS="PARSEC_MCA_device_hip_cu_yield=1" TAG=y bash scripts/gpu/r4_qr_domain.sh || exit 1
