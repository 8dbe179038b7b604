mkdir -p gpurun_out/sp && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
PARSEC_POTRF_SPREAD=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > gpurun_out/sp/kt.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 PARSEC_POTRF_SPREAD=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/sp/k1.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/sp/k0.log 2>&1 &&
bash scripts/gpu/bench_ab.sh "s1a;PARSEC_POTRF_SPREAD=1;--size 16384 --nb 512 --steps 5 --warmup 1" "s0a;;--size 16384 --nb 512 --steps 5 --warmup 1" "s1b;PARSEC_POTRF_SPREAD=1;--size 16384 --nb 512 --steps 5 --warmup 1" "s0b;;--size 16384 --nb 512 --steps 5 --warmup 1"
rc=$?; tail -1 gpurun_out/sp/kt.log; grep -h "us" gpurun_out/sp/k1.log gpurun_out/sp/k0.log | grep -v amdgpu; exit $rc
