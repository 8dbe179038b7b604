#!/bin/bash
# Round 6 validation: the whole GPU suite, smoke(), configs 3 and 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${R6_OUT:-r6v1}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 250 --timeout-method thread > $O/test.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/test.log | head -20; tail -1 $O/test.log
[ $rc -eq 0 ] || [ "${R6_CONTINUE:-0}" = 1 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cut -c1-300 $O/c3.json
timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cut -c1-300 $O/c2.json
exit $rc
