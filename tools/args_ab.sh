#!/bin/bash
# bench.py lines under alternative argument sets, interleaved twice, one line
# each (value, ms/step, copy rates, verified).
# usage: tools/args_ab.sh OUT "ARGS_A" "ARGS_B" ...
set -u
out=$1; shift
: > $out
for r in 1 2; do
  for a in "$@"; do
    res=$(timeout -k 10 300 python bench.py --no-cpu-baseline $a 2>/dev/null) || exit 1
    echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('[$a]', round(d['value'],1), round(d['ms_per_step'],2), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> $out
  done
done
