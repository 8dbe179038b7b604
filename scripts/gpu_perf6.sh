#!/bin/bash
# Manager inline dispatch + bulk-stream batch throttling: 16k and 64k benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { timeout -k 10 600 python bench.py --gpus 1 "$@"; }
timeout -k 10 300 python -u -m pytest tests/test_dpotrf_gpu.py tests/test_dgeqrf.py tests/test_stencil3d.py tests/test_collection_ops.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_eng.log 2>&1 && \
for cfg in "1 2" "1 0" "0 0" "1 4"; do
  set -- $cfg
  for r in 1 2; do run --size 16384 --nb 512 --steps 5 --warmup 2 --mca device_manager_inline_dispatch $1 --mca device_hip_max_inflight_batches $2 > gpurun_out/b16k_i$1_g$2_r$r.log 2>&1 || exit $?; done
done && \
run --steps 3 --warmup 1 > gpurun_out/b64k_i1_g2.log 2>&1 && \
run --steps 3 --warmup 1 --mca device_hip_max_inflight_batches 0 > gpurun_out/b64k_i1_g0.log 2>&1
rc=$?
tail -n 2 gpurun_out/pytest_eng.log
for f in gpurun_out/b16k_i*.log gpurun_out/b64k_i*.log; do echo -n "$f "; grep "^{" $f | python3 -c "import json,sys; [print(d['value'], d['ms_per_step'], d.get('gpu_kernel_launches')) for d in map(json.loads, sys.stdin)]"; done
exit $rc
