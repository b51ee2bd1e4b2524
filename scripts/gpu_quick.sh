# Focused GPU check: named tests first, then the whole GPU suite, then the
# lean-relay timing and a 1-GPU bench line without the CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-q}
if [ -n "$FIRST_TESTS" ]; then
timeout -k 10 300 python -u -m pytest $FIRST_TESTS -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_first_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_first_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_first_$TAG.log
fi
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
fi
if [ -n "$EXTRA" ]; then
timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/extra_$TAG.txt 2>&1 || { tail -30 gpurun_out/extra_$TAG.txt; exit 1; }
tail -40 gpurun_out/extra_$TAG.txt
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
fi
