set -o pipefail
D=gpurun_out/r05steal3; mkdir -p $D
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/honu_amd/libhonu_codec_ab.so
XE="--shape mixed --mode encode --no-cpu-baseline --no-host-path --no-decode-legs --legs none --steps 12 --warmup 3"
prof() {  # tag variant
  if [ $2 = 8 ]; then
    HONU_LIB_PATH=$AB HONU_COPY_VARIANT=43 HONU_COPY_STEAL=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/$1 -o run -- python bench.py $XE > $D/$1.json 2> $D/$1.err
  else
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/$1 -o run -- python bench.py $XE > $D/$1.json 2> $D/$1.err
  fi
}
prof warm 0 || exit $?
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="0 8"; else order="8 0"; fi
  for u in $order; do prof mixenc_s${u}_r$r $u || exit $?; done
done
