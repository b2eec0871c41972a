#!/bin/bash
# Round 6: GPU suite, Small A/B (guard grid, copy order), default line.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c3_tests.log 2>&1 || exit 1
NL="--no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 20 --warmup 5 --shape small"
bash tools/r06_ab.sh gpurun_out/r06_ab_small 3 "$NL" "default:" "guard64:--guard-blocks 64" \
  "guard256:--guard-blocks 256" "ahead3:--copy-order ahead --slots 3" > gpurun_out/r06_ab_small.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_c3_bench.json 2> gpurun_out/r06_c3_bench.err || exit 3
bash tools/r06_ab.sh gpurun_out/r06_ab_zc 2 "--mode decode --decode-leg zero_copy --zc-forms default --no-cpu-baseline --no-host-path --legs none --steps 10" "spec1:" "spec0:--zc-speculate 0" > gpurun_out/r06_ab_zc.log 2>&1 || exit 4
