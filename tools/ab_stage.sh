#!/bin/bash
# Stage timings (tools/meta_sweep.py) of library builds side by side.
# usage: tools/ab_stage.sh SHAPE N tag=path ...   ("cur" = in-tree build)
set -u
shape=$1; n=$2; shift 2
for r in 1 2; do
  for spec in cur=- "$@"; do
    tag=${spec%%=*}; path=${spec#*=}
    if [ "$path" = - ]; then unset HONU_LIB_PATH; else export HONU_LIB_PATH=$path; fi
    timeout -k 10 200 python tools/meta_sweep.py --shape $shape --sizes $n --reps 5 2>/dev/null \
      | python -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$tag', json.dumps(d['us']), 'meta', d['metadata_us'], d['ok'])" || exit 1
  done
done
