# round 6: the GPU suite, then (when green) the default bench line.
# usage: bash tools/r06_gpu_tests.sh [tag] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-t}
shift || true
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r06_$tag.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py "$@" > gpurun_out/r06_${tag}_bench.json 2> gpurun_out/r06_${tag}_bench.err
