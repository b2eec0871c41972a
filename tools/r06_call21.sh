#!/bin/bash
# Round 6 call 21: the window-2 tail-flag check (tools/tmp/tl.so,
# HONU_GATHER_SKIP_WIN2=1) against the product build: parity through the
# variant, zero-copy and materialising timing, FETCH/WRITE of both decodes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_tl
mkdir -p $O
R=$GRAFT_REPO_ROOT
HONU_LIB_PATH=$R/tools/tmp/tl.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 \
  --timeout-method thread tests/test_lookback.py tests/test_gpu_parity.py tests/test_golden_batches.py \
  tests/test_full_size.py > $O/tests.log 2>&1 || exit 1
LIBS=$R/honu_amd/libhonu_codec.so,$R/tools/tmp/tl.so
WL=small:1048576,large:262144
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 9 > $O/zc.jsonl 2> $O/zc.err || exit 2
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 2 --reps 5 --what mat > $O/mat.jsonl 2> $O/mat.err || exit 3
for v in base:honu_amd/libhonu_codec.so tl:tools/tmp/tl.so; do
  tag=${v%%:*}
  export HONU_LIB_PATH=$R/${v#*:}
  tools/pmc_passes.sh $O/pmc_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child \
    --workloads small:1048576,large:262144 --reps 3 > $O/pmc_$tag.log 2>&1 || exit 4
  tools/pmc_passes.sh $O/pmcmat_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child --what mat \
    --workloads small:1048576 --reps 3 > $O/pmcmat_$tag.log 2>&1 || exit 5
done
exit 0
