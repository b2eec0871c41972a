#!/bin/bash
# Round 6 call 17: stream priorities for the Small and Medium lines (copy
# stream high, the default; neither; the metadata streams high), interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
NL="--no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 20 --warmup 5"
bash tools/r06_ab.sh gpurun_out/r06_prio_small 3 "$NL --shape small" "copy_hi:" "none:--copy-prio 0" \
  "meta_hi:--copy-prio -1" > gpurun_out/r06_prio_small.log 2>&1 || exit 1
bash tools/r06_ab.sh gpurun_out/r06_prio_medium 2 "$NL --shape medium" "copy_hi:" "none:--copy-prio 0" \
  "meta_hi:--copy-prio -1" > gpurun_out/r06_prio_medium.log 2>&1 || exit 2
exit 0
