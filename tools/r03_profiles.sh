#!/bin/bash
# Round-3 evidence, each step under its own time limit, stopping at the first
# failure:
#   decode  rocprofv3 --kernel-trace --stats of bench.py --mode decode (the
#           whole-batch zero-copy + materialising decode of 1M Large), and
#           FETCH_SIZE / WRITE_SIZE passes of each leg alone (so a kernel's
#           per-launch traffic belongs to one leg)
#   shapes  FETCH_SIZE / WRITE_SIZE passes of the Medium and XLarge bench lines
#           (no host-path or decode legs, whose launches would mix in)
# usage: tools/r03_profiles.sh OUT decode|shapes
set -u
out=$1; what=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W="1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena"
if [ "$what" = decode ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_decode -o run --output-format csv \
    -- python3 bench.py --mode decode --no-cpu-baseline > $out/bench_decode_prof.json 2> $out/prof_decode.log || exit 1
  cp "$(find $out/prof_decode -name '*kernel_stats.csv' | head -n 1)" $out/kernel_stats_decode.csv
  for leg in zero_copy materialising; do
    tools/pmc_passes.sh $out/pmc_$leg "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --mode decode \
      --decode-leg $leg --no-cpu-baseline > $out/pmc_$leg.log 2>&1 || exit 1
    python3 tools/pmc_traffic.py "$(find $out/pmc_$leg/p1 -name '*counter_collection.csv' | head -n 1)" \
      "$(find $out/pmc_$leg/p2 -name '*counter_collection.csv' | head -n 1)" "$W, $leg" \
      $out/pmc_traffic.json > $out/traffic_$leg.txt || exit 1
  done
fi
if [ "$what" = shapes ]; then
  for spec in medium:1048576 xlarge:65536; do
    shape=${spec%%:*}; n=${spec##*:}
    tools/pmc_passes.sh $out/pmc_$shape "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --shape $shape \
      --records $n --no-cpu-baseline --no-decode-legs --no-host-path > $out/pmc_$shape.log 2>&1 || exit 1
    python3 tools/pmc_traffic.py "$(find $out/pmc_$shape/p1 -name '*counter_collection.csv' | head -n 1)" \
      "$(find $out/pmc_$shape/p2 -name '*counter_collection.csv' | head -n 1)" \
      "$n $shape records per GPU: encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)" \
      $out/pmc_traffic.json > $out/traffic_$shape.txt || exit 1
  done
fi
exit 0
