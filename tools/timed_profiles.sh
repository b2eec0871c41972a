#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench command of each GPU config,
# and the per-kernel statistics of its TIMED steps cut out of the same trace
# (tools/timed_stats.py: the untimed verification step runs digest kernels
# beside the next chunk's copies and slows them, which the whole-process
# --stats average includes). Each step under its own time limit, stopping at
# the first failure.
# usage: tools/timed_profiles.sh OUT [SHAPE...]   (default: large small mixed)
set -u
out=$1; shift
shapes=${*:-large small mixed}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for shape in $shapes; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$shape -o run --output-format csv \
    -- python3 bench.py --shape $shape --no-cpu-baseline > $out/bench_prof_$shape.json 2> $out/prof_$shape.log || exit 1
  tr=$(find $out/prof_$shape -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_$shape -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_$shape.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_$shape.json $out/timed_kernel_stats_$shape.csv \
    > $out/timed_$shape.txt || exit 1
  cat $out/timed_$shape.txt
  gzip -f "$tr"
done
