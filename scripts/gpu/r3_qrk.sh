#!/bin/bash
# Isolated QR tile-kernel latencies and their per-kernel trace
set -o pipefail
mkdir -p gpurun_out/q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 scripts/qr_kbench.py 512 > gpurun_out/q/qrk.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/q/qrk -o run -- python3 scripts/qr_kbench.py 512 > gpurun_out/q/qrk2.log 2>&1
rc=$?; cat gpurun_out/q/qrk.log
f=$(find gpurun_out/q/qrk -name "*kernel_trace.csv" -print -quit)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"])) for r in rows)
# last TSQRT call: find qr_sub2 kernels with 1 WG; print one TSQRT's sequence
sub = [k for k in ks if "qr_sub2" in k[2] or "qr_subapply" in k[2]]
seq = sub[-120:-60]
t0 = seq[0][0]
for s, e, n, g in seq[:40]:
    print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} wg{g:5d} {n}")
PY
exit $rc
