#!/bin/bash
# Counter passes over the zero-copy decode of one workload (tools/decode_ab.py
# child, product library unless HONU_LIB_PATH says otherwise):
#   tools/fused_pmc.sh OUTDIR small:1048576
set -u
out=$1; wl=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/pmc_passes.sh "$out" \
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
  "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
  "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT" \
  "FETCH_SIZE" "WRITE_SIZE" \
  -- python3 tools/decode_ab.py --child --workloads "$wl" --reps 3
