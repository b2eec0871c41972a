#!/bin/bash
# Round 6 call 8: the ACL list's partial end chunks written by the list kernel
# (HONU_ACL_ENDS=1, tools/tmp/ends1.so) against the product build: parity
# through the variant, header/tail encoder timing (tools/decode_ab.py --what
# encode), the Small line, and FETCH/WRITE passes of the encoder child.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_ends
mkdir -p $O
V=$GRAFT_REPO_ROOT/tools/tmp/ends1.so
B=$GRAFT_REPO_ROOT/honu_amd/libhonu_codec.so
HONU_LIB_PATH=$V timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_golden_batches.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/decode_ab.py --what encode --libs $B,$V --workloads small:1048576,large:262144 \
  --rounds 3 --reps 9 > $O/enc.jsonl 2> $O/enc.err || exit 2
for r in 1 2; do
  for v in base:$B ends1:$V; do
    tag=${v%%:*}
    HONU_LIB_PATH=${v#*:} timeout -k 10 300 python3 bench.py --shape small --legs none --no-decode-legs \
      --no-cpu-baseline --no-host-path --steps 20 --warmup 5 > $O/small_${tag}_$r.json 2> $O/small_${tag}_$r.err || exit 3
  done
done
for v in base:$B ends1:$V; do
  tag=${v%%:*}
  export HONU_LIB_PATH=${v#*:}
  tools/pmc_passes.sh $O/pmc_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child --what encode \
    --workloads small:1048576 --reps 3 > $O/pmc_$tag.log 2>&1 || exit 4
done
exit 0
