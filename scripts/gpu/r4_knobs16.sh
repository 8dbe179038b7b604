#!/bin/bash
# Config 2 (16k / nb 512): runtime threads and bulk batching knobs, round-4 engine.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r4_knobs16 bash scripts/gpu/bench_ab.sh \
 "base;;$B" \
 "c8;;$B --cores 8" \
 "c2;;$B --cores 2" \
 "g1;;$B --mca device_hip_group_rounds 1" \
 "g3;;$B --mca device_hip_group_rounds 3" \
 "m1;;$B --mca device_hip_max_inflight_batches 1" \
 "m3;;$B --mca device_hip_max_inflight_batches 3" \
 "base2;;$B" || exit 1
