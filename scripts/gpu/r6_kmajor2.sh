#!/bin/bash
# Round 6: odd-stride k-contiguous LDS rows (BK + 1): tests, LDS conflicts, QR apply rate, configs 4 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/kmaj2; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dgeqrf.py tests/test_headline_gpu.py tests/test_collection_ops.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/q -o run -- python3 benchmarks/bench_workloads.py qr --size 8192 --nb 512 --steps 1 --warmup 0 > $O/q.log 2>&1 || { tail -5 $O/q.log; exit 1; }
f=$(find $O/q -name "*counter_collection.csv" -print -quit); python3 scripts/lds_conflicts.py $f > $O/qr_lds.txt; head -6 $O/qr_lds.txt; rm -rf $O/q
timeout -k 10 200 python3 scripts/kbench_qr_apply.py > $O/k.log 2>&1 || { tail -5 $O/k.log; exit 1; }
grep qr_apply $O/k.log
: > $O/qr.txt
for name in q1 q2 q3; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "$name : $(grep -h '^{' $O/$name.log | cut -c1-140)" >> $O/qr.txt
done
cat $O/qr.txt
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
cut -c1-120 $O/c3.json
