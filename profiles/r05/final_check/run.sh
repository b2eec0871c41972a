set -o pipefail
D=gpurun_out/r05z; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_suite.log 2>&1 || { tail -30 $D/gpu_suite.log; exit 1; }
tail -1 $D/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 2; }
tail -1 $D/smoke.log
timeout -k 10 600 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 3; }
python -c "import json; j=json.load(open('$D/bench_default.json')); print(j['value'], j['roofline']['frac'], j['legs']['small']['ms_per_step'], j['legs']['mixed_encode']['ms_per_step'], j['decode']['zero_copy']['ms'])"
