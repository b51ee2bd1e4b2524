# Wide converge path: parity tests then timings (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-w}
timeout -k 10 400 python -m pytest tests/test_gpu_wide.py -m gpu -v -p no:cacheprovider --timeout 300 > gpurun_out/pytest_wide_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_wide_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_wide_$TAG.log
timeout -k 10 300 python scripts/wide_timing.py > gpurun_out/wide_timing_$TAG.txt 2>&1 || { tail -20 gpurun_out/wide_timing_$TAG.txt; exit 1; }
grep n_dual gpurun_out/wide_timing_$TAG.txt
