#!/bin/bash
# Round 6 call 33: does running the host-path leg first change the main line?
# The main line with the host path first (default) and at the end,
# interleaved, 3 rounds (no other legs).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_hostorder
mkdir -p $O
B="--no-cpu-baseline --no-decode-legs --legs none --steps 20 --warmup 5"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $B > $O/first_r$r.json 2> $O/first_r$r.err || exit 1
  timeout -k 10 300 python bench.py $B --host-path-at end > $O/end_r$r.json 2> $O/end_r$r.err || exit 2
done
