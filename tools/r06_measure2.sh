#!/bin/bash
# Round 6, one GPU call: PMC traffic part 2 (Mixed encode, Medium, XLarge) and
# the copy attribution passes (tools/copy_attr.sh).
# usage: HONU_COMMIT=<sha> bash tools/r06_measure2.sh
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/r06_pmc.sh gpurun_out/r06pmc 2 > gpurun_out/r06pmc_part2.log 2>&1 || exit 1
bash tools/copy_attr.sh gpurun_out/r06attr > gpurun_out/r06attr.log 2>&1 || exit 2
exit 0
