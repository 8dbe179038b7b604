#!/bin/bash
# Round 6: same-box A/B of config 3 between this tree and a build of an earlier commit (_old/, temporary).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/oldnew; mkdir -p $O; : > $O/ab.txt
for spec in new old new old new old; do
  if [ $spec = new ]; then d=.; else d=_old; fi
  timeout -k 10 400 python3 $d/bench.py --steps 3 --warmup 1 > $O/$spec.json 2> $O/$spec.err || { tail -5 $O/$spec.err; exit 1; }
  echo "$spec $(cut -c90-140 $O/$spec.json)" >> $O/ab.txt
done
cat $O/ab.txt
