set -o pipefail
D=gpurun_out/r05steal4; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
C="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
run() {  # tag variant args...
  local tag=$1 u=$2; shift 2
  if [ $u = 8 ]; then HONU_LIB_PATH=$AB HONU_COPY_VARIANT=43 HONU_COPY_STEAL=8 timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err
  else timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err; fi
}
run warm 0 --shape small $C --steps 10 --warmup 3 || exit $?
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 8"; else order="8 0"; fi
  for u in $order; do run small_s${u}_r$r $u --shape small $C --steps 30 --warmup 5 || exit $?; done
  for u in $order; do run medium_s${u}_r$r $u --shape medium $C --steps 10 --warmup 3 || exit $?; done
  for u in $order; do run mix_s${u}_r$r $u --shape mixed $C --steps 8 --warmup 2 || exit $?; done
  for u in $order; do run large_s${u}_r$r $u --shape large $C --steps 4 --warmup 2 || exit $?; done
done
