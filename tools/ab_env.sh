#!/bin/bash
# Interleaved A/B of bench.py under different environment settings on one box.
# usage: tools/ab_env.sh OUT "BENCH ARGS" "ENV1" "ENV2" ...   (ENV "" = defaults)
set -u
out=$1; args=$2; shift 2
: > $out
for r in 1 2; do
  for e in "$@"; do
    res=$(env $e timeout -k 10 300 python bench.py --no-cpu-baseline $args 2>/dev/null) || exit 1
    echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('[$e]', round(d['value'],1), round(d['ms_per_step'],2), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> $out
  done
done
