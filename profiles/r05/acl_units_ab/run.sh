set -o pipefail
D=gpurun_out/r05acl; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
HONU_LIB_PATH=$AB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "encode or acl or pairs" > $D/gpu_ab.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $D/gpu_ab.log; tail -2 $D/gpu_ab.log
[ $rc -eq 0 ] || exit $rc
S="--shape small --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 20 --warmup 5"
SE="--shape small --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 20 --warmup 5"
XE="--shape mixed --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 6 --warmup 2"
run() {  # tag ab args...
  local tag=$1 u=$2; shift 2
  if [ $u = 1 ]; then HONU_LIB_PATH=$AB timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err
  else timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err; fi
}
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 1"; else order="1 0"; fi
  for u in $order; do run small_a${u}_r$r $u $S || exit $?; run smallenc_a${u}_r$r $u $SE || exit $?; done
done
for r in 1 2; do
  if [ $r = 1 ]; then order="0 1"; else order="1 0"; fi
  for u in $order; do run mixenc_a${u}_r$r $u $XE || exit $?; done
done
