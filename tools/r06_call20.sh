#!/bin/bash
# Round 6 call 20: the GPU suite on the committed code, the decode against the
# previous build (tools/tmp/prev.so: before the nt policy and the header
# change), then the PMC passes of part 1. usage: tools/r06_call20.sh COMMIT
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r06_c20_tests.log 2>&1 || exit 1
LIBS=$R/tools/tmp/prev.so,$R/honu_amd/libhonu_codec.so
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads small:1048576,large:262144 --rounds 3 \
  --reps 9 > gpurun_out/r06_c20_zc.jsonl 2> gpurun_out/r06_c20_zc.err || exit 2
HONU_COMMIT=$1 bash tools/r06_pmc.sh gpurun_out/r06pmc8 1 || exit 3
exit 0
