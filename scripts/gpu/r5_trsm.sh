#!/bin/bash
# Round 5: host-decided panel solve (no gated TRSM kernel on the critical stream).
# TRSM-mode GPU test, headline + config 2 bench, config-3 kernel statistics.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trsm
timeout -k 10 300 python3 -u -m pytest tests/test_dpotrf_gpu.py -x -v --timeout 200 --timeout-method thread -k "trsm_inverse or headline or dpotrf" > gpurun_out/trsm/test.log 2>&1 || { tail -40 gpurun_out/trsm/test.log; exit 1; }
tail -3 gpurun_out/trsm/test.log
timeout -k 10 400 python3 bench.py > gpurun_out/trsm/bench64.json 2> gpurun_out/trsm/bench64.err || { tail -20 gpurun_out/trsm/bench64.err; exit 1; }
cut -c1-400 gpurun_out/trsm/bench64.json; grep -o '"panel_solve.*' gpurun_out/trsm/bench64.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/trsm/bench16.json 2> gpurun_out/trsm/bench16.err || { tail -20 gpurun_out/trsm/bench16.err; exit 1; }
cut -c1-300 gpurun_out/trsm/bench16.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trsm/c3 -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/trsm/c3.log 2>&1 || { tail -5 gpurun_out/trsm/c3.log; exit 1; }
f=$(find gpurun_out/trsm/c3 -name "*kernel_stats.csv" -print -quit); cp $f gpurun_out/trsm/c3_kernel_stats.csv
rm -rf gpurun_out/trsm/c3
head -12 gpurun_out/trsm/c3_kernel_stats.csv | cut -c1-160
