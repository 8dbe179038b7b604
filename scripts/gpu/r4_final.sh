#!/bin/bash
# Round-4 validation on the final tree: GPU suite, smoke, headline bench (configs
# 3 and 2), then diagnostics (QR sub-panel phases under load, config-2 knobs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/final/gpu_suite.log 2>&1 || { tail -40 gpurun_out/final/gpu_suite.log; exit 1; }
tail -2 gpurun_out/final/gpu_suite.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench64.json 2> gpurun_out/final/bench64.err || { tail -20 gpurun_out/final/bench64.err; exit 1; }
cut -c1-300 gpurun_out/final/bench64.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/final/bench16.json 2> gpurun_out/final/bench16.err || { tail -20 gpurun_out/final/bench16.err; exit 1; }
cut -c1-300 gpurun_out/final/bench16.json
bash scripts/gpu/r4_qr_phases.sh || exit 1
bash scripts/gpu/r4_knobs16.sh || exit 1
