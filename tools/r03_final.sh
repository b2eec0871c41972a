#!/bin/bash
# Round-3 final evidence of the main bench lines, each step under its own time
# limit, stopping at the first failure:
#   1. rocprofv3 --kernel-trace --stats of bench.py (Large, Small, Mixed) without
#      the host-path and decode legs (their launches of the same kernels would
#      shift the timed window's launch indices), and the stats of the timed
#      steps cut from the same trace (tools/timed_stats.py)
#   2. FETCH_SIZE / WRITE_SIZE passes of the Small line (the metadata kernels
#      changed this round) -> OUT/pmc_traffic.json
# usage: tools/r03_final.sh OUT
set -u
out=$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for shape in large small mixed; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$shape -o run --output-format csv \
    -- python3 bench.py --shape $shape --no-cpu-baseline --no-host-path --no-decode-legs \
    > $out/bench_prof_$shape.json 2> $out/prof_$shape.log || exit 1
  tr=$(find $out/prof_$shape -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_$shape -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_$shape.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_$shape.json $out/timed_kernel_stats_$shape.csv \
    > $out/timed_$shape.txt || exit 1
  gzip -f "$tr"
done
tools/pmc_passes.sh $out/pmc_small "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --shape small \
  --no-cpu-baseline --no-host-path --no-decode-legs > $out/pmc_small.log 2>&1 || exit 1
python3 tools/pmc_traffic.py "$(find $out/pmc_small/p1 -name '*counter_collection.csv' | head -n 1)" \
  "$(find $out/pmc_small/p2 -name '*counter_collection.csv' | head -n 1)" \
  "1048576 small records per GPU: encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)" \
  $out/pmc_traffic.json > $out/traffic_small.txt || exit 1
exit 0
