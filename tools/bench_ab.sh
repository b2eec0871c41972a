#!/bin/bash
# Interleaved bench.py runs of two library builds on one box (process-to-
# process and box-to-box spread hit both alike): OUT_DIR LIB_A LIB_B ROUNDS ARGS...
# one JSON line per run in OUT_DIR/ab.jsonl, tagged with the library.
set -euo pipefail
out=$1; a=$2; b=$3; rounds=$4; shift 4
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in "$a" "$b"; do
    HONU_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python bench.py "$@" --no-cpu-baseline \
        --no-host-path --no-decode-legs > "$out/run.json" 2> "$out/run.err"
    python -c "
import json, sys
d = json.load(open('$out/run.json'))
print(json.dumps({'lib': '$lib', 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'frac': d['roofline']['frac'], 'verified': d['verified'],
                  'zc': d['kernels']['zero_copy_decode_records_per_s']}))" >> "$out/ab.jsonl"
  done
done
