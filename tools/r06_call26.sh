#!/bin/bash
# Round 6 call 26: does the host-path leg (run first, on a fresh device) or the
# decode legs (the 207 GB records arena, run before the shape legs) change the
# main line or the legs after them? The default line (minus the CPU baseline,
# which runs last) against --no-host-path and --no-decode-legs, interleaved,
# 2 rounds.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_order2
mkdir -p $O
B="--no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/default_r$r.json 2> $O/default_r$r.err || exit 1
  timeout -k 10 300 python bench.py $B --no-host-path > $O/nohost_r$r.json 2> $O/nohost_r$r.err || exit 2
  timeout -k 10 300 python bench.py $B --no-decode-legs > $O/nodec_r$r.json 2> $O/nodec_r$r.err || exit 3
done
exit 0
