#!/bin/bash
# Round 6 call 25: is the Small leg slower after the Large line (4.28-4.32 ms)
# than alone (3.94-4.16 ms) because of the order? The default line with the
# Small and XLarge legs after the main line (0) and before it (1, --legs-first),
# interleaved, 2 rounds each, then the Small line alone once.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_legorder
mkdir -p $O
NL="--no-cpu-baseline --no-host-path --no-decode-legs --steps 20 --warmup 5"
for r in 1 2; do
  for f in 0 1; do
    timeout -k 10 300 python bench.py $NL --legs small,xlarge --legs-first $f > $O/f${f}_r$r.json 2> $O/f${f}_r$r.err || exit 1
  done
done
timeout -k 10 200 python bench.py $NL --shape small --legs none > $O/alone.json 2> $O/alone.err || exit 2
exit 0
