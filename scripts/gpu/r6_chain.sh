#!/bin/bash
# Round 6: config-2 critical-chain routes with the one-panel lookahead set
# critical (PARSEC_DPOTRF_SYRK_LOOKAHEAD=3) and the cost of the packed panel tile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_chain bash scripts/gpu/bench_ab.sh \
 "b;;$C2" \
 "np;PARSEC_POTRF_PACK=0;$C2" \
 "la3;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2" \
 "la3h0;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0" \
 "la3h2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3 GPU_MAX_HW_QUEUES=8;$C2 --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" \
 "la3h0r16x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 16 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h0r32x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 32 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h2r32x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3 GPU_MAX_HW_QUEUES=8;$C2 --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4 --mca device_hip_reserved_cus 32 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h0r32;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 32" \
 "b2;;$C2" \
 "np2;PARSEC_POTRF_PACK=0;$C2" || exit 1
# config 4 (1 GPU): the ptgpp-compiled dgeqrf.jdf vs the hand-built flat DAG and
# the round-5 default (hierarchical tree, flat on one process row)
O=gpurun_out/ab; : > $O/r6_qr.txt
for spec in "jdf;--taskpool jdf --qr-tree flat" "ir;--taskpool ir --qr-tree flat" "hqr;--qr-tree hqr" "jdf2;--taskpool jdf --qr-tree flat"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check $args > $O/qr_$name.log 2>&1 || { echo "qr $name failed"; tail -5 $O/qr_$name.log; exit 1; }
  echo "$name $args : $(grep -h '^{' $O/qr_$name.log | cut -c1-400)" >> $O/r6_qr.txt
done
cat $O/r6_qr.txt
