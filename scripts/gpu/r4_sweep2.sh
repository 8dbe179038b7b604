#!/bin/bash
# DGEQRF 32k tile-size sweep (config 4 leaves nb free), then DPOTRF bulk-inflight
# variants: max_inflight_batches 1 vs adaptive critical_bulk_cap 1 at 16k / 64k.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrnb
for nb in 256 384 1024; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb $nb --steps 2 --warmup 1 > gpurun_out/qrnb/$nb.json 2> gpurun_out/qrnb/$nb.err || { tail -5 gpurun_out/qrnb/$nb.err; exit 1; }
  echo "qr32 nb $nb $(cut -c1-130 gpurun_out/qrnb/$nb.json)"
done
B="--size 16384 --nb 512 --steps 5 --warmup 1"
C="--steps 3 --warmup 1"
AB_TAG=r4_inflight2 bash scripts/gpu/bench_ab.sh \
 "m2_16;;$B" "m1_16;;$B --mca device_hip_max_inflight_batches 1" "cc1_16;;$B --mca device_hip_critical_bulk_cap 1" \
 "m2_16b;;$B" "m1_16b;;$B --mca device_hip_max_inflight_batches 1" "cc1_16b;;$B --mca device_hip_critical_bulk_cap 1" \
 "m1_64;;$C --mca device_hip_max_inflight_batches 1" "cc1_64;;$C --mca device_hip_critical_bulk_cap 1" "m2_64;;$C" || exit 1
