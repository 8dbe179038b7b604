#!/bin/bash
# Round-4 validation after the reshape / C API / QR VGPR cap / stencil remap / inflight default
# changes: GPU suite, smoke, headline (config 3), config 2, QR 32k, stencil.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/final2/gpu_suite.log 2>&1 || { tail -40 gpurun_out/final2/gpu_suite.log; exit 1; }
tail -2 gpurun_out/final2/gpu_suite.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/final2/bench64.json 2> gpurun_out/final2/bench64.err || { tail -20 gpurun_out/final2/bench64.err; exit 1; }
cut -c1-300 gpurun_out/final2/bench64.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/final2/bench16.json 2> gpurun_out/final2/bench16.err || { tail -20 gpurun_out/final2/bench16.err; exit 1; }
cut -c1-300 gpurun_out/final2/bench16.json
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/final2/qr32.json 2> gpurun_out/final2/qr32.err || { tail -5 gpurun_out/final2/qr32.err; exit 1; }
cut -c1-200 gpurun_out/final2/qr32.json
timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > gpurun_out/final2/stencil.json 2> gpurun_out/final2/stencil.err || { tail -5 gpurun_out/final2/stencil.err; exit 1; }
cut -c1-200 gpurun_out/final2/stencil.json
