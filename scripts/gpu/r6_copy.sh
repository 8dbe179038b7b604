#!/bin/bash
# Round 6: shared copy stream under host-resident DPOTRF (capped cache /
# fitting cache / two logical devices), engine counters + rocprofv3 memory-copy
# statistics (copy engine busy time against the span).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6copy; mkdir -p $O
for spec in "evict;16384 512 0.25" "fit;16384 512 2.0" "two;16384 512 0.0 2"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 200 python3 scripts/copy_stream_profile.py $args > $O/$name.txt 2>&1 || { echo "$name failed"; tail -5 $O/$name.txt; exit 1; }
  tail -1 $O/$name.txt
  timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/p_$name -o run -- python3 scripts/copy_stream_profile.py $args > $O/p_$name.log 2>&1 || { echo "prof $name failed"; tail -5 $O/p_$name.log; exit 1; }
  f=$(find $O/p_$name -name "*memory_copy_stats.csv" -print -quit); [ -n "$f" ] && cp $f $O/${name}_memcopy_stats.csv
  f=$(find $O/p_$name -name "*kernel_stats.csv" -print -quit); [ -n "$f" ] && cp $f $O/${name}_kernel_stats.csv
  f=$(find $O/p_$name -name "*memory_copy_trace.csv" -print -quit); [ -n "$f" ] && python3 scripts/copy_occupancy.py $f > $O/${name}_occupancy.txt 2>&1
  rm -rf $O/p_$name
  cat $O/${name}_occupancy.txt 2>/dev/null | head -12
done
