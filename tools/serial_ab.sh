set -u
: > gpurun_out/serial_ab.txt
for shape in small medium mixed; do
 for r in 1 2; do
  for m in "" "--serial"; do
    res=$(timeout -k 10 300 python bench.py --no-cpu-baseline --shape $shape $m 2>/dev/null) || exit 1
    echo "$res" | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$shape [$m]', round(d['value'],1), round(d['ms_per_step'],3), 'enc', round(k['encode_copy_gbs']), 'dec', round(k['decode_copy_gbs']), 'frac', round(d['roofline']['frac'],3), d['verified'])" >> gpurun_out/serial_ab.txt
  done
 done
done
