# k_solve_pipe fusing Y'Qd on a launch's first iterate: parity, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_u.log 2>&1 || { tail -40 gpurun_out/pt_u.log; exit 1; }
tail -1 gpurun_out/pt_u.log
timeout -k 10 300 python -u scripts/batch_converge_breakdown.py 1024 4096 4 fused_T,single_T > gpurun_out/bd_u.json 2> gpurun_out/bd_u.err || { tail -20 gpurun_out/bd_u.err; exit 1; }
cat gpurun_out/bd_u.json
