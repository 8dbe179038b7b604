#!/bin/bash
# Round 6 closing profiles: kernel statistics of configs 3 and 2, QR (JDF / IR alternating), stencil.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/fin6; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dpotrf_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p3 -o run -- python3 bench.py --steps 1 --warmup 1 > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
f=$(find $O/p3 -name "*kernel_stats.csv" -print -quit); cp $f $O/kernel_stats_c3.csv; grep -h '^{' $O/p3.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p2 -o run -- python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
f=$(find $O/p2 -name "*kernel_stats.csv" -print -quit); cp $f $O/kernel_stats_c2.csv; grep -h '^{' $O/p2.log | cut -c1-200
rm -rf $O/p3 $O/p2
: > $O/qr.txt
for spec in "ir;--taskpool ir" "jdf;--taskpool jdf" "ir2;--taskpool ir" "jdf2;--taskpool jdf"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check $args > $O/q_$name.log 2>&1 || { tail -5 $O/q_$name.log; exit 1; }
  echo "$name $args : $(grep -h '^{' $O/q_$name.log | cut -c1-160)" >> $O/qr.txt
done
cat $O/qr.txt
timeout -k 10 300 python3 benchmarks/bench_workloads.py stencil > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
grep -h '^{' $O/st.log | cut -c1-200
