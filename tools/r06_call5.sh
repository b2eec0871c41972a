#!/bin/bash
# Round 6 call 5: window alignment A/B of the single-launch decode
# (win.h HONU_WIN_ALIGN 16 / 64 / 128, tools/variant_lib.sh builds of fused.hip):
# zero-copy and materialising timing interleaved (tools/decode_ab.py), then
# FETCH_SIZE / WRITE_SIZE passes of the zero-copy child per build.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_win
mkdir -p $O
LIBS=honu_amd/libhonu_codec.so,tools/tmp/w64.so,tools/tmp/w128.so
WL=small:1048576,large:262144
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 9 > $O/zc.jsonl 2> $O/zc.err || exit 1
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 2 --reps 5 --what mat > $O/mat.jsonl 2> $O/mat.err || exit 2
for v in base:honu_amd/libhonu_codec.so w64:tools/tmp/w64.so w128:tools/tmp/w128.so; do
  tag=${v%%:*}
  export HONU_LIB_PATH=$GRAFT_REPO_ROOT/${v#*:}
  tools/pmc_passes.sh $O/pmc_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child --workloads $WL --reps 3 > $O/pmc_$tag.log 2>&1 || exit 3
done
exit 0
