#!/bin/bash
# Copy-stage timings in isolation (tools/meta_sweep.py) for the short-record
# shapes, default engine and the given ctx params.
set -u
for shape in small medium large; do
  n=1048576; [ $shape = large ] && n=65536
  timeout -k 10 200 python tools/meta_sweep.py --shape $shape --sizes $n --reps 5 --params "${1:-copy_variant=0}" 2>/dev/null \
    | python -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); u=d['us']; print('$shape', d['records'], 'enc_copy', u['encode_copy'], 'dec_copy', u['decode_copy'], 'meta', d['metadata_us'], 'ok', d['ok'])" || exit 1
done
