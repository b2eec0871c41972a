set -o pipefail
D=gpurun_out/r05steal6; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
C="--no-cpu-baseline --no-host-path --no-decode-legs --legs none"
run() {  # tag share args...
  local tag=$1 u=$2; shift 2
  HONU_LIB_PATH=$AB HONU_COPY_VARIANT=45 HONU_COPY_STEAL=$u timeout -k 10 300 python bench.py "$@" > $D/$tag.json 2> $D/$tag.err
}
run warm 8 --shape medium $C --steps 5 --warmup 2 || exit $?
for r in 1 2 3 4; do
  case $r in 1) order="4 8 16 24";; 2) order="24 16 8 4";; 3) order="8 24 4 16";; 4) order="16 4 24 8";; esac
  for u in $order; do run mixenc_s${u}_r$r $u --shape mixed --mode encode $C --steps 12 --warmup 3 || exit $?; done
  for u in $order; do run mix_s${u}_r$r $u --shape mixed $C --steps 8 --warmup 2 || exit $?; done
  for u in $order; do run medium_s${u}_r$r $u --shape medium $C --steps 10 --warmup 3 || exit $?; done
done
