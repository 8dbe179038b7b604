#!/bin/bash
# SYRK(k, k+2) lookahead priority (PARSEC_DPOTRF_SYRK_LOOKAHEAD) at configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AB_TAG=r4_syrk_lookahead bash scripts/gpu/bench_ab.sh \
 "l0_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "l1_16;PARSEC_DPOTRF_SYRK_LOOKAHEAD=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "l0b_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "l1b_16;PARSEC_DPOTRF_SYRK_LOOKAHEAD=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "l0_64;;--steps 2 --warmup 1" \
 "l1_64;PARSEC_DPOTRF_SYRK_LOOKAHEAD=1;--steps 2 --warmup 1" || exit 1
