#!/bin/bash
# Round 6: host-hop components on the config-2 critical stream (kernel trace + launch log in one run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/hoplat; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 --mca device_hip_trace_launches 1 > $O/b.json 2> $O/launch.log || { tail -5 $O/launch.log; exit 1; }
gzip -f $O/launch.log
t=$(find $O/t -name "*kernel_trace.csv" -print -quit)
python3 scripts/hop_latency.py $t $O/launch.log.gz > $O/hops.txt 2>&1; cat $O/hops.txt
gzip -c $t > $O/trace.csv.gz; rm -rf $O/t
