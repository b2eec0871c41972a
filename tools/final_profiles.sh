#!/bin/bash
# The round's committed measurements of the default command, each step under
# its own time limit, stopping at the first failure:
#   1. python bench.py (default: 1M Large, with the CPU baseline)
#   2. rocprofv3 --kernel-trace --stats of the same command
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command -> traffic
#   4. one bench line per README shape
set -u
out=gpurun_out/final
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof -o r01 --output-format csv -- python3 bench.py > $out/prof_bench.log 2>&1 || exit 1
tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --no-cpu-baseline > $out/pmc.log 2>&1 || exit 1
tools/shape_sweep.sh $out/shapes || exit 1
