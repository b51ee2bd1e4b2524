# Split-kernel parity subset + timings (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-q}
timeout -k 10 300 python -m pytest tests/test_gpu_rowshard.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 -k "rowblock or rowshard or synth_rows or split or large_fixed or bundled_fixed" > gpurun_out/pytest_split_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_split_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_split_$TAG.log
timeout -k 10 300 python scripts/single_timing.py > gpurun_out/single_$TAG.txt 2>&1 || { tail -20 gpurun_out/single_$TAG.txt; exit 1; }
tail -1 gpurun_out/single_$TAG.txt
timeout -k 10 300 python scripts/rowshard_timing.py ${RS_ARGS:-} > gpurun_out/rowshard_timing_$TAG.txt 2>&1 || { cat gpurun_out/rowshard_timing_$TAG.txt; exit 1; }
grep n_dual gpurun_out/rowshard_timing_$TAG.txt
