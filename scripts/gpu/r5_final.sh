#!/bin/bash
# Round 5 closing validation: the whole GPU suite, smoke(), every BASELINE config
# on one GPU (3 headline, 2, 4 QR with the R check, 5 stencil, 1 DTD GEMM) and the
# config-3 kernel statistics.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/final5; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/test.log | tail -30; tail -60 $O/test.log | cut -c1-300; exit 1; }
grep -cE "PASSED" $O/test.log; tail -1 $O/test.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cut -c1-300 $O/c3.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cut -c1-300 $O/c2.json
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
cut -c1-300 $O/c4.json
timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cut -c1-300 $O/c5.json
timeout -k 10 200 python3 benchmarks/bench_workloads.py dtd_gemm > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cut -c1-300 $O/c1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p3 -o run -- python3 bench.py --steps 1 --warmup 1 > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
f=$(find $O/p3 -name "*kernel_stats.csv" -print -quit); cp $f $O/c3_kernel_stats.csv; rm -rf $O/p3
head -8 $O/c3_kernel_stats.csv | cut -c1-200
