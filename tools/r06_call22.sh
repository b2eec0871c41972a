#!/bin/bash
# Round 6 call 22 (after the session restart): the GPU suite and the smoke on
# the product build at HEAD, then call 21's window-2 tail-flag A/B
# (tools/tmp/tl.so: HONU_GATHER_SKIP_WIN2=1).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_c22
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
bash tools/r06_call21.sh
