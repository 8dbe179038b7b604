#!/bin/bash
# Round 5 validation 1: host-decided panel solve, fetch queue, copy-engine IPC
# route, superseded DTD versions; headline + config 2; config-3 kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/v1; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_dpotrf_gpu.py tests/test_multirank_gpu.py tests/test_gpu_programs.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/test.log | tail -30; tail -60 $O/test.log | cut -c1-300; exit 1; }
grep -cE "PASSED" $O/test.log; tail -2 $O/test.log
timeout -k 10 400 python3 bench.py > $O/bench64.json 2> $O/bench64.err || { tail -20 $O/bench64.err; exit 1; }
cut -c1-300 $O/bench64.json; grep -o '"panel_solve.*' $O/bench64.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > $O/bench16.json 2> $O/bench16.err || { tail -20 $O/bench16.err; exit 1; }
cut -c1-300 $O/bench16.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 bench.py --steps 1 --warmup 1 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
f=$(find $O/c3 -name "*kernel_stats.csv" -print -quit); cp $f $O/c3_kernel_stats.csv
rm -rf $O/c3
head -12 $O/c3_kernel_stats.csv | cut -c1-160
