set -o pipefail
D=gpurun_out/r05steal5; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_suite.log 2>&1 || { tail -30 $D/gpu_suite.log; exit 1; }
tail -1 $D/gpu_suite.log
HONU_LIB_PATH=$AB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k copy_engine > $D/gpu_ab.log 2>&1 || { tail -30 $D/gpu_ab.log; exit 1; }
tail -1 $D/gpu_ab.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 2
C="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
run() {  # tag variant args...  (variant 1: range tails on, the product; 0: off, A/B variant 44)
  local tag=$1 u=$2; shift 2
  if [ $u = 0 ]; then HONU_LIB_PATH=$AB HONU_COPY_VARIANT=44 timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err
  else timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err; fi
}
run warm 1 --shape small $C --steps 10 --warmup 3 || exit $?
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 1"; else order="1 0"; fi
  for u in $order; do run small_s${u}_r$r $u --shape small $C --steps 30 --warmup 5 || exit $?; done
  for u in $order; do run medium_s${u}_r$r $u --shape medium $C --steps 10 --warmup 3 || exit $?; done
  for u in $order; do run mixenc_s${u}_r$r $u --shape mixed --mode encode $C --steps 12 --warmup 3 || exit $?; done
  for u in $order; do run mix_s${u}_r$r $u --shape mixed $C --steps 8 --warmup 2 || exit $?; done
  for u in $order; do run large_s${u}_r$r $u --shape large $C --steps 4 --warmup 2 || exit $?; done
done
