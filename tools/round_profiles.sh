#!/bin/bash
# The round's committed measurements, per BASELINE config with a GPU line
# (default 1M Large, 1M Small, 1M Mixed), each step under its own time limit,
# stopping at the first failure:
#   1. the bench line (python bench.py [--shape S])
#   2. rocprofv3 --kernel-trace --stats of the same command
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command -> HBM
#      traffic per kernel launch, merged into OUT/pmc_traffic.json by workload
# usage: tools/round_profiles.sh OUT TAG
set -u
out=$1; tag=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cp profiles/pmc_traffic.json $out/pmc_traffic.json 2>/dev/null
for shape in large small mixed; do
  args="--shape $shape"
  cpu=""
  [ $shape = large ] || cpu="--no-cpu-baseline"
  timeout -k 10 400 python bench.py $args $cpu > $out/bench_$shape.json 2> $out/bench_$shape.err || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$shape -o $tag --output-format csv -- python3 bench.py $args --no-cpu-baseline > $out/prof_$shape.log 2>&1 || exit 1
  tools/pmc_passes.sh $out/pmc_$shape "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py $args --no-cpu-baseline > $out/pmc_$shape.log 2>&1 || exit 1
  w=$(python3 -c "import json; print(json.load(open('$out/bench_$shape.json'))['config']['workload'])")
  python3 tools/pmc_traffic.py $out/pmc_$shape/p1/*counter_collection.csv $out/pmc_$shape/p2/*counter_collection.csv "$w" $out/pmc_traffic.json > $out/traffic_$shape.txt || exit 1
done
