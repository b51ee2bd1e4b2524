# k_solve_mid (batched mid-size path): its parity tests, the horizon sweep
# with the path on and off, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mid.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_mid.log 2>&1 || { tail -40 gpurun_out/pt_mid.log; exit 1; }
tail -2 gpurun_out/pt_mid.log
timeout -k 10 300 python -u scripts/horizon_sweep.py ${SWEEP_H:-1 2 3 4 5 6 8} > gpurun_out/horizon_mid.jsonl 2> gpurun_out/horizon_mid.err || { tail -20 gpurun_out/horizon_mid.err; exit 1; }
cat gpurun_out/horizon_mid.jsonl
[ -n "$NO_SUITE" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_all_f.log 2>&1 || { tail -40 gpurun_out/pt_all_f.log; exit 1; }
tail -3 gpurun_out/pt_all_f.log
