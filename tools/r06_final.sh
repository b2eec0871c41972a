#!/bin/bash
# Round-6 final evidence for the code as committed, each step under its own
# time limit, stopping at the first failure. usage: tools/r06_final.sh OUT PART
#   part 1: pytest -m gpu, smoke(), the default bench line (driver command),
#           rocprofv3 --kernel-trace --stats of the Large line with its timed
#           steps cut out (tools/timed_stats.py)
#   part 2: the same for the Small line (pipelined and --serial), and the
#           zero-copy leg's trace
set -u
out=$1; part=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NL="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
trace() {  # name args...: kernel-trace + stats of one bench command, timed window cut out
  local name=$1; shift
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run --output-format csv \
    -- python3 bench.py "$@" > $out/bench_prof_$name.json 2> $out/prof_$name.log || return 1
  local tr st
  tr=$(find $out/prof_$name -name '*kernel_trace.csv' | head -n 1)
  st=$(find $out/prof_$name -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_$name.csv
  python3 tools/timed_stats.py "$tr" $out/bench_prof_$name.json $out/timed_kernel_stats_$name.csv \
    > $out/timed_$name.txt || return 2
  gzip -f "$tr"
}
if [ "$part" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $out/gpu_suite.log 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 2
  t0=$(date +%s.%N)
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_default.json 2> $out/bench_default.err || exit 3
  t1=$(date +%s.%N)
  python3 -c "print('bench.py --steps 20 --warmup 5 wall time: %.1f s' % ($t1 - $t0))" > $out/bench_default_wall.txt
  trace large $NL || exit 4
fi
if [ "$part" = 2 ]; then
  trace small --shape small --steps 20 --warmup 5 $NL || exit 1
  # the same with one stream (no copy beside the metadata kernels): how much
  # the pipeline stretches each metadata kernel
  trace small_serial --shape small --serial --steps 20 --warmup 5 $NL || exit 3
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_zc -o run --output-format csv \
    -- python3 bench.py --mode decode --decode-leg zero_copy --zc-forms default --steps 10 --no-cpu-baseline \
    --no-host-path --legs none > $out/bench_prof_zc.json 2> $out/prof_zc.log || exit 2
  st=$(find $out/prof_zc -name '*kernel_stats.csv' | head -n 1)
  cp "$st" $out/kernel_stats_zc.csv
  gzip -f "$(find $out/prof_zc -name '*kernel_trace.csv' | head -n 1)"
fi
exit 0
