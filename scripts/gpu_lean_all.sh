# lean form: its tests, then the timelines and the A/B (scripts/gpu_lean_trace.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06g}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_persist_lean.py > gpurun_out/pytest_lean_$T.log 2>&1 || { tail -30 gpurun_out/pytest_lean_$T.log; exit 1; }
tail -2 gpurun_out/pytest_lean_$T.log
TAG=$T bash scripts/gpu_lean_trace.sh
