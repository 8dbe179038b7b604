#!/bin/bash
# Headline re-check: bench.py defaults (config 3) twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rc64
for i in 1 2; do
  timeout -k 10 400 python3 bench.py > gpurun_out/rc64/b$i.json 2> gpurun_out/rc64/b$i.err || { tail -20 gpurun_out/rc64/b$i.err; exit 1; }
  echo "b64 $i $(cut -c80-150 gpurun_out/rc64/b$i.json)"
done
