#!/bin/bash
# Config 2 (16k / nb 512): manager launch timeline + rocprofv3 kernel trace of
# the same run shape, for the per-panel critical-chain analysis.
set -o pipefail
mkdir -p gpurun_out/${T16:-t16}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PARSEC_MCA_device_hip_trace_launches=1 timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 2 --warmup 1 $EXTRA > gpurun_out/${T16:-t16}/bench.json 2> gpurun_out/${T16:-t16}/launches.log || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T16:-t16}/prof -o run -- python3 bench.py --size 16384 --nb 512 --steps 2 --warmup 1 $EXTRA > gpurun_out/${T16:-t16}/prof.log 2>&1 || exit 1
f=$(find gpurun_out/${T16:-t16}/prof -name "*kernel_trace.csv" -print -quit)
python3 scripts/critical_chain.py $f 512 16384 > gpurun_out/${T16:-t16}/chain16.txt
cp $f gpurun_out/${T16:-t16}/kernel_trace.csv
gzip -f gpurun_out/${T16:-t16}/kernel_trace.csv gpurun_out/${T16:-t16}/launches.log
rm -rf gpurun_out/${T16:-t16}/prof
head -3 gpurun_out/${T16:-t16}/chain16.txt; tail -1 gpurun_out/${T16:-t16}/chain16.txt; cat gpurun_out/${T16:-t16}/bench.json | cut -c1-200
