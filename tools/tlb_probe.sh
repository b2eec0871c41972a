#!/bin/bash
set -u
# TLB counters of the copy kernels under three separate bench processes
# (tests whether the between-process spread is address translation).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tlb
for p in 1 2 3; do
  timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum GRBM_UTCL2_BUSY -d gpurun_out/tlb/p$p -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 > gpurun_out/tlb/p$p.log 2>&1 || exit 1
done
