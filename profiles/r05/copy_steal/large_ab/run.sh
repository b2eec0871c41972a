set -o pipefail
D=gpurun_out/r05large; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
C="--shape large --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 6 --warmup 2"
run() {  # tag variant (1: range tails on, the product; 0: off, A/B variant 44)
  if [ $2 = 0 ]; then HONU_LIB_PATH=$AB HONU_COPY_VARIANT=44 timeout -k 10 300 python bench.py $C > $D/$1.json 2> $D/$1.err
  else timeout -k 10 300 python bench.py $C > $D/$1.json 2> $D/$1.err; fi
}
run warm 1 || exit $?
for r in 1 2 3 4 5 6; do
  if [ $((r % 2)) = 1 ]; then order="0 1"; else order="1 0"; fi
  for u in $order; do run large_s${u}_r$r $u || exit $?; done
done
