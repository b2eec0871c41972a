#!/bin/bash
# Round 6 call 13: the flag burst's window skip in the speculative decode too
# (tools/tmp/gs2w64.so: HONU_GATHER_SKIP_WIN=1 HONU_WIN_ALIGN=64) against the
# product build and gs1w64: parity through the variant, zero-copy and
# materialising timing, the Small line, FETCH/WRITE of both decodes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_gs2
mkdir -p $O
R=$GRAFT_REPO_ROOT
B=$R/honu_amd/libhonu_codec.so
V=$R/tools/tmp/gs2w64.so
HONU_LIB_PATH=$V timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_lookback.py tests/test_gpu_parity.py tests/test_golden_batches.py tests/test_full_size.py \
  tests/test_bench_decode.py > $O/tests.log 2>&1 || exit 1
LIBS=$B,$R/tools/tmp/gs1w64.so,$V
WL=small:1048576,large:262144
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 9 > $O/zc.jsonl 2> $O/zc.err || exit 2
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 5 --what mat > $O/mat.jsonl 2> $O/mat.err || exit 3
for r in 1 2; do
  for v in base:$B gs2w64:$V; do
    tag=${v%%:*}
    HONU_LIB_PATH=${v#*:} timeout -k 10 300 python3 bench.py --shape small --legs none --no-decode-legs \
      --no-cpu-baseline --no-host-path --steps 20 --warmup 5 > $O/small_${tag}_$r.json 2> $O/small_${tag}_$r.err || exit 4
  done
done
for v in base:$B gs2w64:$V; do
  tag=${v%%:*}
  export HONU_LIB_PATH=${v#*:}
  tools/pmc_passes.sh $O/pmc_mat_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child --what mat \
    --workloads small:1048576 --reps 3 > $O/pmc_mat_$tag.log 2>&1 || exit 5
done
exit 0
