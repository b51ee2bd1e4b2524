# Row-shard tests, full GPU suite, and split-kernel timing/profile (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-rs}
timeout -k 10 300 python -m pytest tests/test_gpu_rowshard.py -m gpu -v -p no:cacheprovider --timeout 200 > gpurun_out/pytest_rowshard_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_rowshard_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_rowshard_$TAG.log
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python scripts/rowshard_timing.py > gpurun_out/rowshard_timing_$TAG.txt 2>&1 || { cat gpurun_out/rowshard_timing_$TAG.txt; exit 1; }
cat gpurun_out/rowshard_timing_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_single_$TAG -o single -- python3 scripts/single_timing.py > gpurun_out/single_$TAG.txt 2>&1 || { tail -20 gpurun_out/single_$TAG.txt; exit 1; }
tail -2 gpurun_out/single_$TAG.txt
