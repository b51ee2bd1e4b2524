# configs[2] lean (one-XCD) form: its tests, the split form's tests and the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06d}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_persist_lean.py tests/test_gpu_persist.py tests/test_gpu_persist_fit.py > gpurun_out/pytest_lean_$T.log 2>&1 && timeout -k 10 120 python scripts/persist_lean_ab.py 5 > gpurun_out/persist_lean_ab_$T.json 2> gpurun_out/persist_lean_ab_$T.err
rc=$?
tail -3 gpurun_out/pytest_lean_$T.log; cat gpurun_out/persist_lean_ab_$T.json; exit $rc
