set -o pipefail
D=gpurun_out/r05steal; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
if [ -z "$SKIP_TESTS" ]; then
  HONU_LIB_PATH=$AB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "copy_engine" > $D/gpu_ab.log 2>&1 || exit $?
fi
XE="--shape mixed --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 6 --warmup 2"
X="--shape mixed --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 4 --warmup 2"
L="--shape large --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 4 --warmup 2"
run() {  # tag variant args...
  local tag=$1 u=$2; shift 2
  case $u in
    0) timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err ;;
    8) HONU_LIB_PATH=$AB HONU_COPY_VARIANT=43 HONU_COPY_STEAL=8 timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err ;;
    16) HONU_LIB_PATH=$AB HONU_COPY_VARIANT=43 HONU_COPY_STEAL=16 timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err ;;
  esac
}
D=gpurun_out/r05steal2; mkdir -p $D
XE="--shape mixed --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 12 --warmup 3"
run warm 0 $XE || exit $?
for r in 1 2 3 4 5 6; do
  if [ $((r % 2)) = 1 ]; then order="0 8"; else order="8 0"; fi
  for u in $order; do run mixenc_s${u}_r$r $u $XE || exit $?; done
done
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 8"; else order="8 0"; fi
  for u in $order; do run mix_s${u}_r$r $u $X || exit $?; done
done
