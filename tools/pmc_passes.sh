#!/bin/bash
# Run one rocprofv3 counter pass per argument group ("A B C" ...) over the
# command after "--", each pass under its own time limit. Stops at the first
# pass that times out, aborts or faults; a pass whose counters cannot be
# collected together just reports and the next pass runs.
# usage: tools/pmc_passes.sh OUTDIR "CNT1 CNT2" "CNT3" -- cmd args...
set -u
out=$1; shift
passes=()
while [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
mkdir -p "$out"
k=0
for p in "${passes[@]}"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --pmc $p -d "$out/p$k" -o run --output-format csv -- "$@" > "$out/p$k.log" 2>&1
  rc=$?
  echo "pass $k [$p] rc=$rc"
  case $rc in 124|137|134|139) echo "stopping"; exit $rc;; esac
done
