set -o pipefail
D=gpurun_out/r05short; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
HONU_LIB_PATH=$AB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "copy_engine and (short_tails or no_tails or steal_off or default)" > $D/gpu_ab.log 2>&1 || { tail -20 $D/gpu_ab.log; exit 1; }
tail -1 $D/gpu_ab.log
XE="--shape mixed --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 12 --warmup 3"
X="--shape mixed --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 8 --warmup 2"
run() {  # tag variant args...
  local tag=$1 u=$2; shift 2
  HONU_LIB_PATH=$AB HONU_COPY_VARIANT=$u timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err
}
run warm 0 $XE || exit $?
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 46"; else order="46 0"; fi
  for u in $order; do run mixenc_s${u}_r$r $u $XE || exit $?; done
  for u in $order; do run mix_s${u}_r$r $u $X || exit $?; done
done
