#!/bin/bash
# Interleaved A/B of bench.py argument sets: R rounds, every variant once per
# round (the order rotated per round), one JSON line per run in OUT/ab.jsonl
# ({"tag", "round", "line": the bench line}). Each run under its own limit.
# usage: tools/r06_ab.sh OUT R "common args" "tag1:args1" "tag2:args2" ...
set -u
out=$1; R=$2; common=$3; shift 3
mkdir -p $out
cd "$GRAFT_REPO_ROOT"
vars=("$@")
nv=${#vars[@]}
for r in $(seq 1 $R); do
  for k in $(seq 0 $((nv - 1))); do
    v=${vars[$(( (k + r) % nv ))]}
    tag=${v%%:*}; args=${v#*:}
    timeout -k 10 300 python3 bench.py $common $args > $out/run.json 2> $out/run_${tag}_$r.err
    rc=$?
    if [ $rc != 0 ]; then echo "run $tag round $r rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac; continue; fi
    python3 -c "import json,sys; l=open('$out/run.json').read().strip().splitlines()[-1]; print(json.dumps({'tag': '$tag', 'round': $r, 'line': json.loads(l)}))" >> $out/ab.jsonl
    echo "round $r $tag done"
  done
done
