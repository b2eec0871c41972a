#!/bin/bash
# Stage times (tools/meta_sweep.py) of the A/B library under settings of one
# environment knob, interleaved twice ("-" = unset).
# usage: tools/env_ab.sh VAR SHAPE SIZES VALUE...   e.g. HONU_FUSED_WIN large 61845 16 32
set -u
var=$1; shape=$2; sizes=$3; shift 3
export HONU_LIB_PATH=honu_amd/libhonu_codec_ab.so
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = - ]; then unset $var; else export $var=$v; fi
    timeout -k 10 300 python tools/meta_sweep.py --shape $shape --sizes $sizes --reps 7 2>/dev/null \
      | python -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); u=d['us']; print('$var=$v', d['records'], 'fused_zc', u.get('fused_zc'), 'fused_mat', u.get('fused_mat'), 'parse', u.get('parse'), 'tables', u.get('tables'), d['ok'])" || exit 1
  done
done
