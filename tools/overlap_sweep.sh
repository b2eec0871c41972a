#!/bin/bash
# Overlap of metadata kernels and payload copies on short records: bench.py
# over copy-engine grid x metadata-kernel caps x chunk counts (no CPU leg).
# usage: tools/overlap_sweep.sh SHAPE OUTFILE
set -u
shape=$1; out=$2
: > $out
for cb in 1 2; do
  for lb in 0 1 2 4; do
    for mc in 4 8; do
      r=$(timeout -k 10 120 python bench.py --shape $shape --no-cpu-baseline --steps 5 --copy-blocks $cb --lane-blocks $lb --min-chunks $mc 2>/dev/null) || exit 1
      echo "$r" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('cb=$cb lb=$lb mc=$mc', round(d['value'],1), 'GiB/s', round(d['ms_per_step'],3), 'ms', 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> $out
    done
  done
done
