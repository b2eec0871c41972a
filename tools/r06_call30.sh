#!/bin/bash
# Round 6 call 30: the PMC traffic passes of the Mixed encode, Medium and
# XLarge lines (tools/r06_pmc.sh part 2, into the part-1 table of call 29),
# then the bench GPU tests at HEAD.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_pmcall2
mkdir -p $O
cp tools/tmp/pmc_part1.json $O/pmc_traffic.json
bash tools/r06_pmc.sh $O 2 || exit $?
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_bench_launcher.py \
  tests/test_bench_legs.py tests/test_bench_decode.py tests/test_bench_pipeline.py > $O/bench_tests.log 2>&1 || exit 9
exit 0
