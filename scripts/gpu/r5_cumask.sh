#!/bin/bash
# CU reservation A/B with the reserved CUs spread over the XCDs (stride 1: CU
# mask bits are dealt to the 8 XCDs round robin) and the bulk GEMM round sized
# to the CUs the bulk streams keep (PARSEC_GEMM_SLOTS = 2 x bulk CUs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/cumask; mkdir -p $O
run() {  # tag size nb steps R stride excl
  local tag=$1 n=$2 nb=$3 st=$4 r=$5 s=$6 x=$7
  local slots=$((2 * (256 - r)))
  PARSEC_MCA_device_hip_reserved_cus=$r PARSEC_MCA_device_hip_reserved_cus_stride=$s PARSEC_MCA_device_hip_reserved_cus_exclusive=$x \
    PARSEC_GEMM_SLOTS=$slots timeout -k 10 300 python3 bench.py --size $n --nb $nb --steps $st --warmup 2 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }
  echo "$tag R=$r stride=$s excl=$x : $(cut -c1-120 $O/$tag.json)"
}
run c2_r0a 16384 512 6 0 1 0 &&
run c2_r8 16384 512 6 8 1 0 &&
run c2_r16 16384 512 6 16 1 0 &&
run c2_r32 16384 512 6 32 1 0 &&
run c2_r16x 16384 512 6 16 1 1 &&
run c2_r0b 16384 512 6 0 1 0 &&
run c3_r0 65536 1024 4 0 1 0 &&
run c3_r8 65536 1024 4 8 1 0 &&
run c3_r16 65536 1024 4 16 1 0
