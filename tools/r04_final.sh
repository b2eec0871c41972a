#!/bin/bash
# Round-4 final evidence, each step under its own time limit, stopping at the
# first failure. usage: tools/r04_final.sh OUT PART
#   part 1: pytest -m gpu, smoke(), the default bench line, rocprofv3
#           --kernel-trace --stats of the Large and Small lines with the timed
#           steps cut from the same trace (tools/timed_stats.py), FETCH_SIZE /
#           WRITE_SIZE passes of the default command (-> pmc_traffic.json) and
#           one TA / TD / TCP pass of it (the copy kernels' L1 path)
#   part 2: FETCH_SIZE / WRITE_SIZE of the configs[2] zero-copy decode leg, and
#           one bench line per README shape
#   part 3 (after the line-drain tail encoder): the Small line's kernel-trace
#           stats and timed steps, FETCH_SIZE / WRITE_SIZE / TA / TD of the
#           tail encoder launched alone on 1M Small (tools/enc_timing.py)
set -u
out=$1; part=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W="1048576 large records per GPU: encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)"
if [ "$part" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $out/gpu_suite.log 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 2
  timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 3
  for shape in large small; do
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$shape -o run --output-format csv \
      -- python3 bench.py --shape $shape --no-cpu-baseline --no-host-path --no-decode-legs \
      > $out/bench_prof_$shape.json 2> $out/prof_$shape.log || exit 4
    tr=$(find $out/prof_$shape -name '*kernel_trace.csv' | head -n 1)
    st=$(find $out/prof_$shape -name '*kernel_stats.csv' | head -n 1)
    cp "$st" $out/kernel_stats_$shape.csv
    python3 tools/timed_stats.py "$tr" $out/bench_prof_$shape.json $out/timed_kernel_stats_$shape.csv \
      > $out/timed_$shape.txt || exit 5
    gzip -f "$tr"
  done
  tools/pmc_passes.sh $out/pmc_large "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
    -- python3 bench.py --no-cpu-baseline --no-host-path --no-decode-legs > $out/pmc_large.log 2>&1 || exit 6
  python3 tools/pmc_traffic.py "$(find $out/pmc_large/p1 -name '*counter_collection.csv' | head -n 1)" \
    "$(find $out/pmc_large/p2 -name '*counter_collection.csv' | head -n 1)" "$W" $out/pmc_traffic.json \
    > $out/traffic_large.txt || exit 7
fi
if [ "$part" = 2 ]; then
  tools/pmc_passes.sh $out/pmc_large2 "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
    -- python3 bench.py --no-cpu-baseline --no-host-path --no-decode-legs > $out/pmc_large2.log 2>&1 || exit 4
  tools/pmc_passes.sh $out/pmc_zc "FETCH_SIZE" "WRITE_SIZE" \
    -- python3 bench.py --mode decode --decode-leg zero_copy --no-cpu-baseline --no-host-path > $out/pmc_zc.log 2>&1 || exit 1
  timeout -k 10 400 python bench.py --mode decode --decode-leg zero_copy --no-cpu-baseline --no-host-path \
    > $out/bench_zero_copy.json 2> $out/bench_zero_copy.err || exit 2
  tools/shape_sweep.sh $out/shapes || exit 3
fi
if [ "$part" = 3 ]; then
  timeout -k 10 300 python bench.py --shape small > $out/bench_small.json 2> $out/bench_small.err || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_small -o run --output-format csv \
    -- python3 bench.py --shape small --no-cpu-baseline --no-host-path --no-decode-legs \
    > $out/bench_prof_small.json 2> $out/prof_small.log || exit 2
  tr=$(find $out/prof_small -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_small -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_small.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_small.json $out/timed_kernel_stats_small.csv \
    > $out/timed_small.txt || exit 3
  gzip -f "$tr"
  tools/pmc_passes.sh $out/pmc_encoder "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
    -- python3 tools/enc_timing.py --shape small --records 1048576 --no-stamps > $out/pmc_encoder.log 2>&1 || exit 4
fi
exit 0
