#!/bin/bash
# IPC pull A/B on 2 shared-GPU ranks (config-2 shape): copy engine vs copy
# kernel, 1 vs 2 pull streams, with per-edge latencies; then a DGEQRF 16k
# kernel profile.
set -o pipefail
mkdir -p gpurun_out/p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
out=gpurun_out/p/pull_ab.txt; : > $out
port=29570
for cfg in "0 1" "0 2" "1 1" "1 2"; do
  set -- $cfg; port=$((port+1))
  PARSEC_MCA_profile_filename=$GRAFT_REPO_ROOT/gpurun_out/p/m$1s$2 PARSEC_MCA_comm_ipc_copy_mode=$1 PARSEC_MCA_comm_ipc_streams=$2 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
     bench.py --gpus 2 --size 16384 --nb 512 --steps 3 --warmup 1 --share-gpu --cores 3 > gpurun_out/p/m$1s$2.log 2>&1 || exit 1
  echo "copy_mode=$1 streams=$2 $(grep -h '^{' gpurun_out/p/m$1s$2.log | cut -c90-140)" >> $out
  python3 scripts/comm_edges.py gpurun_out/p/m$1s$2 2 | grep -E "pull |bandwidth" >> $out
  rm -f gpurun_out/p/m$1s$2-*.prof
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/qr16 -o run -- python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 1 > gpurun_out/p/qr16.log 2>&1
rc=$?
cat $out; grep -h '^{' gpurun_out/p/qr16.log | cut -c1-200
f=$(find gpurun_out/p/qr16 -name "*kernel_stats.csv" -print -quit); [ -n "$f" ] && head -20 $f | cut -d, -f1-6
f=$(find gpurun_out/p/qr16 -name "*kernel_trace.csv" -print -quit); [ -n "$f" ] && python3 scripts/trace_summary.py $f > gpurun_out/p/qr16_summary.txt; head -20 gpurun_out/p/qr16_summary.txt
exit $rc
