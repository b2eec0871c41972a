#!/bin/bash
# A/B of builds of the library on the same box, interleaved (tag=path; "cur"
# is the in-tree build):
# usage: tools/ab_lib.sh OUT "ARGS" tagA=pathA tagB=pathB ...
set -u
out=$1; args=$2; shift 2
: > $out
for r in 1 2; do
  for spec in cur=- "$@"; do
    tag=${spec%%=*}; path=${spec#*=}
    if [ "$path" = - ]; then unset HONU_LIB_PATH; else export HONU_LIB_PATH=$path; fi
    res=$(timeout -k 10 300 python bench.py --no-cpu-baseline $args 2>/dev/null) || exit 1
    echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$tag', round(d['value'],1), round(d['ms_per_step'],2), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), d['verified'])" >> $out
  done
done
