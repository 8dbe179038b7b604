#!/bin/bash
# Full GPU test suite (one pytest process) + smoke
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r3/suite.log 2>&1
rc=$?
grep -E "PASSED|FAILED|SKIPPED|ERROR" gpurun_out/r3/suite.log | tail -100 > gpurun_out/r3/suite_summary.txt
tail -5 gpurun_out/r3/suite.log
[ $rc -eq 0 ] && timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1; rc2=$?
cat gpurun_out/r3/smoke.log 2>/dev/null | tail -2
exit $((rc + rc2))
