#!/bin/bash
# One bench line per README shape (Small/Medium/Large/XLarge + the Mixed
# batch of SURVEY §8d) at N=1, each under its own time limit; stops at the
# first failure. XLarge runs 65,536 records (≈206 GB of payload, the same
# resident footprint as 1M Large); the others 1M records.
# usage: tools/shape_sweep.sh OUTDIR [extra bench args...]
set -u
out=$1; shift
mkdir -p "$out"
for spec in small:1048576 medium:1048576 large:1048576 xlarge:65536 mixed:1048576; do
  shape=${spec%%:*}; n=${spec##*:}
  timeout -k 10 300 python bench.py --shape "$shape" --records "$n" --cpu-seconds 8 "$@" \
    > "$out/$shape.json" 2> "$out/$shape.err"
  rc=$?
  echo "$shape rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
