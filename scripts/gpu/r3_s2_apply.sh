#!/bin/bash
# QR apply as three fused grouped GEMMs (Cin / C2 / a_lower): kernel + QR tests,
# QR benches, DPOTRF no-regression, CU-reservation A/B at 16k, oracle probe.
set -o pipefail
mkdir -p gpurun_out/s3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest --maxfail=4 -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dgeqrf.py tests/test_multirank_gpu.py -k "gemm or qr or dgeqrf or comm_engine" > gpurun_out/s3/tests.log 2>&1
rc0=$?
tail -3 gpurun_out/s3/tests.log; grep -E "FAILED|ERROR" gpurun_out/s3/tests.log | head -10
[ $rc0 -le 1 ] &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --qr-tree flat --check > gpurun_out/s3/qr16_flat.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --check > gpurun_out/s3/qr16_hqr0.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --check > gpurun_out/s3/qr32_hqr0.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 > gpurun_out/s3/b64.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/s3/b16.log 2>&1 &&
for cfg in "8 32" "16 16" "32 8"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 --mca device_hip_reserved_cus $1 --mca device_hip_reserved_cus_stride $2 > gpurun_out/s3/cu_$1_$2.log 2>&1 || exit 1
done &&
timeout -k 10 200 python3 scripts/oracle_probe.py --procs 4 --mode none > gpurun_out/s3/oracle_none.log 2>&1 &&
timeout -k 10 200 python3 scripts/oracle_probe.py --procs 4 --mode init > gpurun_out/s3/oracle_init.log 2>&1
rc=$?
grep -h '^{' gpurun_out/s3/*.log | cut -c1-330; for f in gpurun_out/s3/cu_*.log; do echo "$f $(grep -ho '"value": [0-9.]*' $f)"; done; cat gpurun_out/s3/oracle_*.log | grep proc
exit $((rc0 + rc))
