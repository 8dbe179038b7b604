#!/bin/bash
# Cold-start repeats of the 2-rank GPU QR: fresh process pairs, bad R tiles printed,
# the full logs of a failing run kept (write-back trace on).
mkdir -p gpurun_out
: > gpurun_out/qrcold.log
for i in $(seq 1 ${RUNS:-16}); do
  d=/tmp/qrc$$_$i; mkdir -p $d; J=qc$$_$i
  timeout -k 10 120 env PARSEC_MCA_ptg_trace_writeback=1 python -u tests/mp/gpu_dist.py dgeqrf 0 2 $J 2048 256 2 $d > $d/r0.log 2>&1 &
  p0=$!
  timeout -k 10 120 env PARSEC_MCA_ptg_trace_writeback=1 python -u tests/mp/gpu_dist.py dgeqrf 1 2 $J 2048 256 2 $d > $d/r1.log 2>&1
  r1=$?
  wait $p0; r0=$?
  echo "run $i rc $r0 $r1" >> gpurun_out/qrcold.log
  grep -h "bad" $d/r0.log $d/r1.log >> gpurun_out/qrcold.log
  if grep -q "bad R" $d/r0.log $d/r1.log; then cp $d/r0.log gpurun_out/qrbad_${i}_r0.log; cp $d/r1.log gpurun_out/qrbad_${i}_r1.log; fi
  rm -rf $d
  if [ $r0 -ge 124 ] || [ $r1 -ge 124 ]; then echo "stopping: rc $r0 $r1" >> gpurun_out/qrcold.log; break; fi
done
grep -c "bad R" gpurun_out/qrcold.log
exit 0
