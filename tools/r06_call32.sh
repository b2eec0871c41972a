#!/bin/bash
# Round 6 call 32: one more sample of the driver's command on a fresh box
# (box-to-box spread of the final line).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_c32
mkdir -p $O
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
