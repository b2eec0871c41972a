#!/bin/bash
# Round 6 call 28: the driver's command on a fresh box with the shape legs
# before the decode legs (the new default), first thing in the call, then the
# same with the old order (--legs-at end) as the second process.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_c28
mkdir -p $O
t0=$(date +%s.%N)
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
t1=$(date +%s.%N)
python3 -c "print('bench.py --steps 20 --warmup 5 wall time: %.1f s' % ($t1 - $t0))" > $O/bench_default_wall.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --legs-at end > $O/bench_end.json 2> $O/bench_end.err || exit 2
exit 0
