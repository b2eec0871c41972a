#!/bin/bash
# Round 6 call 6: does the Small leg's step time depend on the load before it?
# The Small leg after the Large line (as in the default line), the same with
# the device idle 10 s before the leg, and Small alone; interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
C="--steps 20 --warmup 5 --no-cpu-baseline --no-host-path"
bash tools/r06_ab.sh gpurun_out/r06_legpause 2 "$C" "after:--legs small" "pause10:--legs small --leg-pause 10" \
  "alone:--shape small --legs none --no-decode-legs" > gpurun_out/r06_legpause.log 2>&1 || exit 1
exit 0
