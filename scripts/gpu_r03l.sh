# k_solve_pipe default build: parity, then the batched converge evidence
# (breakdown pipe vs k_solve_single, kernel trace, FETCH/WRITE passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_pipe3.log 2>&1 || { tail -40 gpurun_out/pt_pipe3.log; exit 1; }
tail -1 gpurun_out/pt_pipe3.log
VARIANTS=fused_T,single_T TAG=${TAG:-bc6} bash scripts/gpu_batch_converge.sh
