#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE passes (tools/pmc_passes.sh) of every
# workload the bench line looks up in profiles/pmc_traffic.json, each entry
# recorded with the commit measured (HONU_COMMIT, from the caller: the box has
# no .git). usage: HONU_COMMIT=<sha> tools/r06_pmc.sh OUT PART
#   part 1: the default Large line, the configs[2] zero-copy and materialising
#           legs, the Small line
#   part 2: the Mixed encode, Medium and XLarge lines
set -u
out=$1; part=$2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NL="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
T=$out/pmc_traffic.json
[ -f $T ] || cp profiles/pmc_traffic.json $T
traffic() {  # dir workload
  python3 tools/pmc_traffic.py "$(find $1/p1 -name '*counter_collection.csv' | head -n 1)" \
    "$(find $1/p2 -name '*counter_collection.csv' | head -n 1)" "$2" $T > $1.txt
}
ED="encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)"
run() {  # name workload args...
  local name=$1 wl=$2; shift 2
  tools/pmc_passes.sh $out/$name "FETCH_SIZE" "WRITE_SIZE" -- python3 bench.py "$@" > $out/$name.log 2>&1 || return 1
  traffic $out/$name "$wl"
}
if [ "$part" = 1 ]; then
  run pmc_large "1048576 large records per GPU: $ED" $NL || exit 1
  run pmc_zc "1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena, zero_copy" \
    --mode decode --decode-leg zero_copy --zc-forms default --no-cpu-baseline --no-host-path --legs none || exit 2
  run pmc_mat "1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena, materialising" \
    --mode decode --decode-leg materialising --no-cpu-baseline --no-host-path --legs none || exit 3
  run pmc_small "1048576 small records per GPU: $ED" --shape small $NL || exit 4
fi
if [ "$part" = 3 ]; then  # the decode legs only (the kernels a decode-only change touches)
  run pmc_zc "1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena, zero_copy" \
    --mode decode --decode-leg zero_copy --zc-forms default --no-cpu-baseline --no-host-path --legs none || exit 2
  run pmc_mat "1048576 large records per GPU: decode (Object.Metadata + Object.Data) of one resident records arena, materialising" \
    --mode decode --decode-leg materialising --no-cpu-baseline --no-host-path --legs none || exit 3
fi
if [ "$part" = 2 ]; then
  run pmc_mixenc "1048576 mixed records per GPU: encode (object.Marshal)" --shape mixed --mode encode $NL || exit 1
  run pmc_medium "1048576 medium records per GPU: $ED" --shape medium $NL || exit 2
  run pmc_xlarge "65536 xlarge records per GPU: $ED" --shape xlarge --records 65536 $NL || exit 3
fi
exit 0
