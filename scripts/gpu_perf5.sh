#!/bin/bash
# W = L^-1 by doubling + diag LDS union: numerics, benches, kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_kern.log 2>&1 && \
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 --check > gpurun_out/b16k_check.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/b16k.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/b64k.log 2>&1 && \
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 \
    bench.py --gpus 2 --size 4096 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 3 > gpurun_out/multi2s.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/p16k -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/prof/bench16k.log 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_kern.log; grep -v amdgpu gpurun_out/kbench.log | grep potrf
for f in gpurun_out/b16k_check.log gpurun_out/b16k.log gpurun_out/b64k.log gpurun_out/multi2s.log gpurun_out/prof/bench16k.log; do echo "== $f"; grep "^{" $f | python3 -c "import json,sys; [print(d['value'], d['ms_per_step'], d.get('max_rel_error_vs_torch_cholesky'), d.get('gpu_kernel_launches')) for d in map(json.loads, sys.stdin)]"; done
exit $rc
