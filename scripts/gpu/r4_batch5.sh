#!/bin/bash
set -o pipefail
bash scripts/gpu/r4_qr_phases.sh || exit 1
bash scripts/gpu/r4_knobs16.sh || exit 1
