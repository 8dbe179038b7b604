#!/bin/bash
# Repeat the 2-rank GPU QR (IPC plane) in one pair of processes and report bad R tiles.
set -o pipefail
mkdir -p gpurun_out /tmp/qrd$$
J=qrd$$
for r in 0 1; do
  timeout -k 10 240 env REPEAT=${REPEAT:-12} python -u tests/mp/gpu_dist.py dgeqrf $r 2 $J 2048 256 2 /tmp/qrd$$ > gpurun_out/qrd_$r.log 2>&1 &
done
wait
rc=$?
tail -n 8 gpurun_out/qrd_0.log gpurun_out/qrd_1.log
exit $rc
