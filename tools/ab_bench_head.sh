#!/bin/bash
# Interleaved A/B of the working-tree bench.py against the committed one:
#   git show HEAD:bench.py > bench_head.py && tools/ab_bench_head.sh (on the GPU box)
set -u
: > gpurun_out/ab_x.txt
for r in 1 2; do
 for shape in small medium large; do
  for b in bench.py bench_head.py; do  # bench_head.py: git show HEAD:bench.py
    res=$(timeout -k 10 300 python $b --no-cpu-baseline --shape $shape 2>/dev/null) || exit 1
    echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$shape $b', round(d['value'],1), round(d['ms_per_step'],3), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> gpurun_out/ab_x.txt
  done
 done
done
