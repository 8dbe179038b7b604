#!/bin/bash
# Round 6: DGEQRF engine knobs again after the conflict-free TN / NN GEMMs (same box, alternating).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qrk6; mkdir -p $O; : > $O/ab.txt
for spec in "b;" "pc2;PARSEC_MCA_device_hip_bulk_gemm_per_cu=2" "m3;PARSEC_MCA_device_hip_max_inflight_batches=3" "gr4;PARSEC_MCA_device_hip_group_rounds=4" \
            "b2;" "pc2b;PARSEC_MCA_device_hip_bulk_gemm_per_cu=2" "m3b;PARSEC_MCA_device_hip_max_inflight_batches=3" "gr4b;PARSEC_MCA_device_hip_group_rounds=4" "b3;"; do
  IFS=';' read -r name envs <<< "$spec"
  env X=1 $envs timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "$name [$envs] $(grep -h '^{' $O/$name.log | cut -c60-100)" >> $O/ab.txt
done
cat $O/ab.txt
