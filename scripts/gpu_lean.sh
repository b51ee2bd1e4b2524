# Lean relay: parity tests then timings (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-l}
timeout -k 10 400 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_rowshard.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_lean_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_lean_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_lean_$TAG.log
timeout -k 10 300 python -u scripts/lean_timing.py > gpurun_out/lean_timing_$TAG.txt 2>&1 || { tail -20 gpurun_out/lean_timing_$TAG.txt; exit 1; }
grep n_dual gpurun_out/lean_timing_$TAG.txt
