#!/bin/bash
# Round 6 call 4: the GPU suite on the speculate-auto default, then the PMC
# passes of part 1 (tools/r06_pmc.sh) for the committed code.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r06_c14_tests.log 2>&1 || exit 1
HONU_COMMIT=$1 bash tools/r06_pmc.sh gpurun_out/r06pmc6 1 || exit 2
exit 0
