#!/bin/bash
# Round 6 call 19: nt (evict-first) cache policy on the decode's window
# refills (ntw) and also its flag bursts (ntall), so that the lines read twice
# (a record's last line = the next record's header line) stay in the L2:
# zero-copy / materialising timing interleaved, FETCH/WRITE passes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_nt
mkdir -p $O
R=$GRAFT_REPO_ROOT
LIBS=$R/honu_amd/libhonu_codec.so,$R/tools/tmp/ntw.so,$R/tools/tmp/ntall.so
WL=small:1048576,large:262144
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 3 --reps 9 > $O/zc.jsonl 2> $O/zc.err || exit 1
timeout -k 10 600 python3 tools/decode_ab.py --libs $LIBS --workloads $WL --rounds 2 --reps 5 --what mat > $O/mat.jsonl 2> $O/mat.err || exit 2
for v in base:honu_amd/libhonu_codec.so ntw:tools/tmp/ntw.so ntall:tools/tmp/ntall.so; do
  tag=${v%%:*}
  export HONU_LIB_PATH=$R/${v#*:}
  tools/pmc_passes.sh $O/pmc_$tag "FETCH_SIZE" "WRITE_SIZE" -- python3 tools/decode_ab.py --child \
    --workloads small:1048576,large:262144 --reps 3 > $O/pmc_$tag.log 2>&1 || exit 3
done
exit 0
