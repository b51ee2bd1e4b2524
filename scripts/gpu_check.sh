# GPU parity tests + smoke + a short bench (run on the GPU box via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "start $(date)"
PYTHONUNBUFFERED=1 timeout -k 10 700 python -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3 --cpu-seconds 10} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
