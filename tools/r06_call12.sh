#!/bin/bash
# Round 6 call 12: the decode's ACL flag burst without the lines the lane's
# window already holds (HONU_GATHER_SKIP_WIN=1), alone and with 64-byte window
# bases (HONU_WIN_ALIGN=64), against the product build: parity through the
# variants, zero-copy / materialising timing interleaved, FETCH/WRITE passes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_gs
mkdir -p $O
R=$GRAFT_REPO_ROOT
for v in gs1 gs1w64; do
  HONU_LIB_PATH=$R/tools/tmp/$v.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 \
    --timeout-method thread tests/test_lookback.py tests/test_gpu_parity.py tests/test_golden_batches.py \
    > $O/tests_$v.log 2>&1 || exit 1
done
LIBS=$R/honu_amd/libhonu_codec.so,$R/tools/tmp/gs1.so,$R/tools/tmp/w64.so,$R/tools/tmp/gs1w64.so
WL=small:1048576,large:262144
timeout -k 10 700 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 9 > $O/zc.jsonl 2> $O/zc.err || exit 2
for v in base:honu_amd/libhonu_codec.so gs1:tools/tmp/gs1.so w64:tools/tmp/w64.so gs1w64:tools/tmp/gs1w64.so; do
  tag=${v%%:*}
  export HONU_LIB_PATH=$R/${v#*:}
  tools/pmc_passes.sh $O/pmc_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child \
    --workloads small:1048576 --reps 3 > $O/pmc_$tag.log 2>&1 || exit 3
done
exit 0
