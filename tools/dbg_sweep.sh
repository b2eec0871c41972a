#!/bin/bash
set -u
for d in ${DBGS:-0 1 2 3}; do
  HONU_FUSED_DBG=$d timeout -k 10 120 python3 tools/meta_sweep.py --shape $1 --sizes $2 --reps 5 > gpurun_out/dbg_$1_$d.jsonl 2>&1 || exit 1
done
