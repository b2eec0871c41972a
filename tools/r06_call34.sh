#!/bin/bash
# Round 6 call 34: the two-rank rehearsal of the whole N > 1 line (host path,
# main line, shape legs, scatter, decode legs) on one GPU, and the launcher tests.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_rehearsal
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_bench_launcher.py \
  > $O/tests.log 2>&1 || exit 1
