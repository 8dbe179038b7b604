#!/bin/bash
# Confirm the LDS padding of bulk GEMMs (rocprofv3 LDS_Block_Size per queue) and
# repeat the per-CU A/B
set -o pipefail
mkdir -p gpurun_out/pc2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pc2/ab.txt; : > $out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pc2/t -o run -- python3 bench.py --size 8192 --nb 512 --steps 1 --warmup 0 --mca device_hip_bulk_gemm_per_cu 1 > gpurun_out/pc2/t.log 2>&1 || exit 1
f=$(find gpurun_out/pc2/t -name "*kernel_trace.csv" -print -quit)
python3 - "$f" <<'PY' >> $out
import csv, sys, collections
c = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "dgemm_batch_kernel<128" in r["Kernel_Name"]:
        c[(r["Queue_Id"], r["LDS_Block_Size"])] += 1
print("128x128 GEMM dispatches by (queue, LDS bytes):", dict(c))
PY
rm -f $f
run() { local n=$1; shift
  timeout -k 10 240 python3 bench.py "$@" > gpurun_out/pc2/$n.log 2>&1 || return 1
  echo "$n $* $(grep -h '^{' gpurun_out/pc2/$n.log | cut -c90-150)" >> $out; }
for i in 1 2; do
  run 16_c2_$i --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_bulk_gemm_per_cu 2 || exit 1
  run 16_c1_$i --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1 || exit 1
done
run 64_c1 --steps 3 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1 && run 64_c2 --steps 3 --warmup 1 --mca device_hip_bulk_gemm_per_cu 2
rc=$?; cat $out; exit $rc
