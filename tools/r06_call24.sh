#!/bin/bash
# Round 6 final evidence, call B: tools/r06_final.sh part 2 (the Small line's
# timed traces, pipelined and serial, and the zero-copy leg's trace), then the
# copy-engine idle gaps of the Small line's timed steps (tools/step_timeline.py).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_final
bash tools/r06_final.sh $O 2 || exit $?
for v in small small_serial; do
  tr=$(find $O/prof_$v -name '*kernel_trace.csv.gz' | head -n 1)
  python3 tools/step_timeline.py "$tr" $O/bench_prof_$v.json 2 > $O/timeline_$v.txt || exit 5
done
exit 0
