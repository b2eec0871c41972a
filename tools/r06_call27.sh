#!/bin/bash
# Round 6 call 27: the order of the line's legs. The default (host path first,
# shape legs at the end) against the shape legs right after the main line
# (before the decode legs' 207 GB records arena), and that with the host path
# at the end too; interleaved, 2 rounds (CPU baseline off: it runs last).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_order3
mkdir -p $O
B="--no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/default_r$r.json 2> $O/default_r$r.err || exit 1
  timeout -k 10 300 python bench.py $B --legs-at after_main > $O/am_r$r.json 2> $O/am_r$r.err || exit 2
  timeout -k 10 300 python bench.py $B --legs-at after_main --host-path-at end > $O/amhe_r$r.json 2> $O/amhe_r$r.err || exit 3
done
exit 0
