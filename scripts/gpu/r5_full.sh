#!/bin/bash
# Round 5 full validation: the whole GPU suite, smoke(), headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/test.log | tail -30; tail -60 $O/test.log | cut -c1-300; exit 1; }
grep -cE "PASSED" $O/test.log; tail -2 $O/test.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench64.json 2> $O/bench64.err || { tail -20 $O/bench64.err; exit 1; }
cut -c1-400 $O/bench64.json
