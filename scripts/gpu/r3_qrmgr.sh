#!/bin/bash
# Manager event log of DGEQRF 16k (flat TS) for the panel-chain analysis
set -o pipefail
mkdir -p gpurun_out/q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PARSEC_MCA_device_hip_trace_launches=1 timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 1 > gpurun_out/q/qrmgr.log 2> gpurun_out/q/qrmgr.err
rc=$?; grep -h '^{' gpurun_out/q/qrmgr.log | cut -c1-150; grep -c engine gpurun_out/q/qrmgr.err; exit $rc
