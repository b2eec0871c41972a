#!/bin/bash
# bench.py over chunk counts x one/two streams for short-record shapes.
set -u
out=$1; : > $out
for shape in small medium mixed; do
  for mc in 1 2 4; do
    for m in "" "--serial"; do
      res=$(timeout -k 10 300 python bench.py --no-cpu-baseline --shape $shape --min-chunks $mc $m 2>/dev/null) || exit 1
      echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$shape mc=$mc [$m]', d['config']['chunks'], round(d['value'],1), round(d['ms_per_step'],3), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> $out
    done
  done
done
