#!/bin/bash

# Round 6: packed panel tile written in POTRF's last launch (validation + cost
# at config 2), configs 3 and 4 (JDF vs IR QR taskpools).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6v2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py tests/test_headline_gpu.py tests/test_dgeqrf.py -m gpu -v -p no:cacheprovider --timeout 250 --timeout-method thread > $O/test.log 2>&1 || { grep -E "FAILED|ERROR" $O/test.log | head; tail -30 $O/test.log | cut -c1-300; exit 1; }
tail -1 $O/test.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_pack bash scripts/gpu/bench_ab.sh "b;;$C2" "np;PARSEC_POTRF_PACK=0;$C2" "b2;;$C2" "np2;PARSEC_POTRF_PACK=0;$C2" "b3;;$C2" "c3;;--steps 3 --warmup 1" || exit 1
: > $O/qr.txt
for spec in "jdf;--taskpool jdf --qr-tree flat" "ir;--taskpool ir --qr-tree flat" "jdf2;--taskpool jdf --qr-tree flat" "ir2;--taskpool ir --qr-tree flat"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check $args > $O/qr_$name.log 2>&1 || { echo "qr $name failed"; tail -5 $O/qr_$name.log; exit 1; }
  echo "$name $args : $(grep -h '^{' $O/qr_$name.log | cut -c1-200) $(grep -ho 'residual[^,]*' $O/qr_$name.log)" >> $O/qr.txt
done
cat $O/qr.txt

# Round 6: shared copy stream under host-resident DPOTRF (capped cache /
# fitting cache / two logical devices), engine counters + rocprofv3 memory-copy
# statistics (copy engine busy time against the span).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6copy; mkdir -p $O
for spec in "evict;16384 512 0.25" "fit;16384 512 2.0" "two;16384 512 0.0 2"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 200 python3 scripts/copy_stream_profile.py $args > $O/$name.txt 2>&1 || { echo "$name failed"; tail -5 $O/$name.txt; exit 1; }
  tail -1 $O/$name.txt
  timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/p_$name -o run -- python3 scripts/copy_stream_profile.py $args > $O/p_$name.log 2>&1 || { echo "prof $name failed"; tail -5 $O/p_$name.log; exit 1; }
  f=$(find $O/p_$name -name "*memory_copy_stats.csv" -print -quit); [ -n "$f" ] && cp $f $O/${name}_memcopy_stats.csv
  f=$(find $O/p_$name -name "*kernel_stats.csv" -print -quit); [ -n "$f" ] && cp $f $O/${name}_kernel_stats.csv
  f=$(find $O/p_$name -name "*memory_copy_trace.csv" -print -quit); [ -n "$f" ] && python3 scripts/copy_occupancy.py $f > $O/${name}_occupancy.txt 2>&1
  rm -rf $O/p_$name
  cat $O/${name}_occupancy.txt 2>/dev/null | head -12
done
# 256 x 128 GEMM macro tiles: kernel rate, then config 3
O=gpurun_out/r6gemm; mkdir -p $O
for v in 0 13 14; do
  PARSEC_GEMM_PAD_TEST=1 PARSEC_GEMM_VARIANT=$v timeout -k 10 200 python3 scripts/kbench_gemm.py > $O/k$v.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/k$v.txt; exit 1; }
  cat $O/k$v.txt
done
AB_TAG=r6_gemm bash scripts/gpu/bench_ab.sh "c3v0;;--steps 3 --warmup 1" "c3v13;PARSEC_GEMM_VARIANT=13;--steps 3 --warmup 1" "c3v14;PARSEC_GEMM_VARIANT=14;--steps 3 --warmup 1" || exit 1
