#!/bin/bash
# Round-5 final evidence, each step under its own time limit, stopping at the
# first failure. usage: tools/r05_final.sh OUT PART
#   part 1: pytest -m gpu, smoke(), the default bench line (Large legs +
#           small + mixed_encode), rocprofv3 --kernel-trace --stats of the
#           Large line with its timed steps cut from the same trace
#           (tools/timed_stats.py), FETCH_SIZE / WRITE_SIZE passes of it
#           (-> profiles/pmc_traffic.json via tools/pmc_traffic.py)
#   part 2: FETCH_SIZE / WRITE_SIZE of the configs[2] zero-copy leg and of the
#           small / mixed_encode leg commands (their workloads' entries in
#           pmc_traffic.json), the Small line's kernel-trace stats and timed
#           steps
set -u
out=$1; part=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NL="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
T=$out/pmc_traffic.json
[ -f $T ] || cp profiles/pmc_traffic.json $T
traffic() {  # dir workload
  python3 tools/pmc_traffic.py "$(find $1/p1 -name '*counter_collection.csv' | head -n 1)" \
    "$(find $1/p2 -name '*counter_collection.csv' | head -n 1)" "$2" $T > $1.txt
}
if [ "$part" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $out/gpu_suite.log 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 2
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || exit 3
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_large -o run --output-format csv \
    -- python3 bench.py $NL > $out/bench_prof_large.json 2> $out/prof_large.log || exit 4
  tr=$(find $out/prof_large -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_large -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_large.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_large.json $out/timed_kernel_stats_large.csv \
    > $out/timed_large.txt || exit 5
  gzip -f "$tr"
  tools/pmc_passes.sh $out/pmc_large "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py $NL > $out/pmc_large.log 2>&1 || exit 6
  traffic $out/pmc_large "1048576 large records per GPU: encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)" || exit 7
fi
if [ "$part" = 2 ]; then
  tools/pmc_passes.sh $out/pmc_zc "FETCH_SIZE" "WRITE_SIZE" \
    -- python3 bench.py --mode decode --decode-leg zero_copy --no-cpu-baseline --no-host-path --legs none > $out/pmc_zc.log 2>&1 || exit 1
  traffic $out/pmc_zc "1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena, zero_copy" || exit 2
  tools/pmc_passes.sh $out/pmc_small "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --shape small $NL > $out/pmc_small.log 2>&1 || exit 3
  traffic $out/pmc_small "1048576 small records per GPU: encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)" || exit 4
  tools/pmc_passes.sh $out/pmc_mixenc "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --shape mixed --mode encode $NL > $out/pmc_mixenc.log 2>&1 || exit 5
  traffic $out/pmc_mixenc "1048576 mixed records per GPU: encode (object.Marshal)" || exit 6
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_small -o run --output-format csv \
    -- python3 bench.py --shape small --steps 20 --warmup 5 $NL > $out/bench_prof_small.json 2> $out/prof_small.log || exit 7
  tr=$(find $out/prof_small -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_small -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_small.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_small.json $out/timed_kernel_stats_small.csv \
    > $out/timed_small.txt || exit 8
  gzip -f "$tr"
fi
exit 0
