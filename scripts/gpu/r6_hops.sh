#!/bin/bash
# Round 6: host hops on the config-2 chain from the manager launch log.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/hops; mkdir -p $O
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 --mca device_hip_trace_launches 1 > $O/b.json 2> $O/launch.log || { tail -5 $O/launch.log; exit 1; }
gzip -f $O/launch.log
python3 scripts/chain_from_launch_log.py $O/launch.log.gz > $O/hops.txt 2>&1; cat $O/hops.txt
