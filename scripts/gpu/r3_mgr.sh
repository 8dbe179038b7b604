#!/bin/bash
# Manager event log (launch / retire / incoming, us timestamps) of config 2
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PARSEC_BENCH_VERBOSE=1 timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 --mca device_hip_trace_launches 1 > gpurun_out/r3/mgr16.log 2> gpurun_out/r3/mgr16.err
rc=$?; grep -h '^{' gpurun_out/r3/mgr16.log | cut -c1-120; grep -c engine gpurun_out/r3/mgr16.err; exit $rc
