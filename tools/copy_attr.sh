#!/bin/bash
# the decode payload copy's counters in three settings,
# one rocprofv3 --pmc pass per counter group (tools/pmc_passes.sh):
#   pipe   the default 1M Large encdec step (the copy beside the metadata
#          kernels of the next chunk, meta_beside decode; no legs)
#   alone  the same chunk's decode copy launched back to back with nothing
#          beside it, then the library's probe copies (NT and default policy)
#          over the same bytes (tools/copy_alone.py)
# then tools/copy_attr.py summarises every setting.
# usage: tools/copy_attr.sh OUT
set -u
out=$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
G1="FETCH_SIZE"
G2="WRITE_SIZE"
G3="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum GRBM_GUI_ACTIVE"
G4="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_CYCLE_sum"
G5="TCC_EA0_WRREQ_STALL_sum TCC_BUSY_sum TCC_CYCLE_sum TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
timeout -k 10 200 python3 tools/copy_alone.py > $out/alone_plain.json 2> $out/alone_plain.err || exit 1
tools/pmc_passes.sh $out/alone "$G1" "$G2" "$G3" "$G4" "$G5" -- python3 tools/copy_alone.py > $out/alone.log 2>&1 || exit 2
tools/pmc_passes.sh $out/pipe "$G1" "$G2" "$G3" "$G4" "$G5" -- python3 bench.py --no-cpu-baseline --no-host-path \
  --no-decode-legs --legs none > $out/pipe.log 2>&1 || exit 3
python3 tools/copy_attr.py $out/alone $out/pipe > $out/summary.json || exit 4
exit 0
