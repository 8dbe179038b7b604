#!/bin/bash
set -o pipefail
bash scripts/gpu/r4_stagger.sh || exit 1
bash scripts/gpu/r4_qr_trace.sh || exit 1
bash scripts/gpu/trace64.sh || exit 1
bash scripts/gpu/r4_syrkla.sh || exit 1
