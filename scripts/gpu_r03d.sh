# converge-mode A/B of two library builds (infeasible and all-feasible
# iterates) and the converge parity tests on the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_converge.py tests/test_gpu_persist_fit.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_d.log 2>&1 || { tail -30 gpurun_out/pt_d.log; exit 1; }
tail -2 gpurun_out/pt_d.log
echo "== infeasible"; ROUNDS=3 bash scripts/converge_ab.sh "$@" || exit 1
echo "== all feasible"; CONVERGE_AB_FEASIBLE=1 ROUNDS=3 bash scripts/converge_ab.sh "$@" || exit 1
