#!/bin/bash
# Round-5 baseline: headline (config 3) and config 2 on the round-4 engine.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/base
timeout -k 10 400 python3 bench.py > gpurun_out/base/bench64.json 2> gpurun_out/base/bench64.err || { tail -20 gpurun_out/base/bench64.err; exit 1; }
cut -c1-300 gpurun_out/base/bench64.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/base/bench16.json 2> gpurun_out/base/bench16.err || { tail -20 gpurun_out/base/bench16.err; exit 1; }
cut -c1-300 gpurun_out/base/bench16.json
