#!/bin/bash
# Round 6: the gfx950 byte-exact memory-side counters (TCC_EA0_RDREQ_*_32B:
# one 32-byte unit per count, a 64-byte request counted twice and a 128-byte
# one four times; TCC_EA0_WRREQ_WRITE_*_32B likewise) beside FETCH_SIZE and the
# request-size counters, over the zero-copy decode bench (whose encode copies
# and probe kernels have known byte counts: the calibration) and the Small line.
# usage: tools/r06_dram_pmc.sh OUT
set -u
out=$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_IO_32B_sum"
P2="TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"
NL="--no-cpu-baseline --no-host-path --legs none"
tools/pmc_passes.sh $out/zc "$P1" "$P2" "$P3" "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --mode decode \
  --decode-leg zero_copy --zc-forms default $NL > $out/zc.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/zc > $out/zc.txt || exit 2
tools/pmc_passes.sh $out/small "$P1" "$P2" "$P3" "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py --shape small \
  --no-decode-legs $NL > $out/small.log 2>&1 || exit 3
python3 tools/pmc_summary.py $out/small > $out/small.txt || exit 4
exit 0
