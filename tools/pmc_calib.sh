#!/bin/bash
# Request-size breakdown of the L2's memory-side reads for the single-launch
# decode (zero copy) and the payload copy, to calibrate FETCH_SIZE for the
# decode's access pattern (MI355X_MICROARCH.md: FETCH_SIZE's x2 correction is
# calibrated for 16-byte-per-lane streaming reads only). One run per counter
# set; tools/decode_ab.py --child runs in-process (no child process under the
# profiler).   tools/pmc_calib.sh OUT_DIR
set -euo pipefail
out=$(realpath -m "$1"); mkdir -p "$out"
root=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$out/$name" -o run -- \
        python3 "$root/tools/decode_ab.py" --child --workloads small:1048576 --reps 3 --what mat \
        > "$out/$name.log" 2>&1
}
run sizes TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
run dram TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
