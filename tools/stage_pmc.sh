#!/bin/bash
# Every codec stage launched alone (tools/meta_sweep.py) with its kernel time
# and, in two separate rocprofv3 PMC passes, its HBM traffic per launch.
# usage: tools/stage_pmc.sh OUTDIR SHAPE RECORDS
set -u
out=$1; shape=$2; n=$3
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/meta_sweep.py --shape "$shape" --sizes "$n" --reps 5 > "$out/sweep.jsonl" 2> "$out/sweep.err" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 tools/meta_sweep.py --shape "$shape" --sizes "$n" --reps 2 > "$out/trace.log" 2>&1 || exit 1
tools/pmc_passes.sh "$out/pmc" "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/meta_sweep.py --shape "$shape" --sizes "$n" --reps 1 > "$out/pmc.log" 2>&1 || exit 1
python3 tools/pmc_traffic.py "$out"/pmc/p1/*/run_counter_collection.csv "$out"/pmc/p2/*/run_counter_collection.csv "meta_sweep $shape $n" "$out/traffic.json" > "$out/traffic.txt"
