#!/bin/bash
# DPOTRF GEMM priority A/B (PARSEC_DPOTRF_GEMM_PRIO: 1 = by column, 0 = DPLASMA
# row order) at configs 2 and 3, plus a config-2 kernel trace -> critical chain
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/gprio_ab.txt; : > $out
run() {  # name, env, args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 240 python3 bench.py "$@" > gpurun_out/r3/gp_$n.log 2>&1 || return 1
  echo "$n $e $* $(grep -h '^{' gpurun_out/r3/gp_$n.log | cut -c90-140)" >> $out
}
run 16_p1 PARSEC_DPOTRF_GEMM_PRIO=1 --size 16384 --nb 512 --steps 4 --warmup 1 &&
run 16_p0 PARSEC_DPOTRF_GEMM_PRIO=0 --size 16384 --nb 512 --steps 4 --warmup 1 &&
run 16_p1_hp0 PARSEC_DPOTRF_GEMM_PRIO=1 --size 16384 --nb 512 --steps 4 --warmup 1 --mca device_hip_hp_on_critical_stream 0 &&
run 16_p1_b PARSEC_DPOTRF_GEMM_PRIO=1 --size 16384 --nb 512 --steps 4 --warmup 1 &&
run 64_p1 PARSEC_DPOTRF_GEMM_PRIO=1 --steps 2 --warmup 1 &&
run 64_p0 PARSEC_DPOTRF_GEMM_PRIO=0 --steps 2 --warmup 1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16b -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/t16b.log 2>&1
rc=$?
cat $out
f=$(find gpurun_out/r3/t16b -name "*kernel_trace.csv" -print -quit); [ -n "$f" ] && python3 scripts/critical_chain.py $f 512 16384 > gpurun_out/r3/chain16b.txt; tail -34 gpurun_out/r3/chain16b.txt
exit $rc
