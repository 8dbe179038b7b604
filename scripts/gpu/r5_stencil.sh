#!/bin/bash
# Round 5: stencil (config 5) bytes per sweep from PMC counters, the practical
# HBM ceiling (streaming copy / read), and the current rate.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/st5; mkdir -p $O
timeout -k 10 120 python3 scripts/copy_bw.py > $O/copy_bw.txt 2>&1 || { tail -5 $O/copy_bw.txt; exit 1; }
cat $O/copy_bw.txt
timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > $O/base.json 2> $O/base.err || { tail -5 $O/base.err; exit 1; }
cut -c1-140 $O/base.json
i=0
for P in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 4 > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
for f in $(find $O -name "*counter_collection.csv"); do python3 scripts/pmc_summary.py $f stencil7v; done > $O/pmc.txt 2>&1
cat $O/pmc.txt
