#!/bin/bash
# GPU variants of the ported reference GPU programs (tests/test_gpu_programs.py)
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_programs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3/progs.log 2>&1
rc=$?
tail -30 gpurun_out/r3/progs.log
exit $rc
