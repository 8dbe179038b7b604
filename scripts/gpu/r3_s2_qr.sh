#!/bin/bash
# Hierarchical QR on the GPU (tests + flat/hqr benches), the CE GPU test, the
# critical-path kernel latencies and a kernel-stats profile of config 2.
set -o pipefail
mkdir -p gpurun_out/s2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest --maxfail=4 -v --timeout 120 --timeout-method thread -m gpu tests/test_dgeqrf.py tests/test_multirank_gpu.py tests/test_dpotrf_gpu.py -k "hqr or comm_engine or redistribute or dgeqrf" > gpurun_out/s2/qr_tests.log 2>&1
rc0=$?
tail -3 gpurun_out/s2/qr_tests.log; grep -E "FAILED|ERROR" gpurun_out/s2/qr_tests.log | head -10
[ $rc0 -le 1 ] &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --qr-tree flat --check > gpurun_out/s2/qr16_flat.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --qr-domain 2 --check > gpurun_out/s2/qr16_hqr2.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --qr-domain 4 --check > gpurun_out/s2/qr16_hqr4.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --qr-domain 8 --check > gpurun_out/s2/qr16_hqr8.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --qr-domain 4 --check > gpurun_out/s2/qr32_hqr4.log 2>&1 &&
timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/s2/kcrit.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/p16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/s2/p16.log 2>&1
rc=$?
cat gpurun_out/s2/kcrit.log; grep -h '^{' gpurun_out/s2/qr*.log | cut -c1-420
exit $((rc0 + rc))
