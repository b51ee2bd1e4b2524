# Round 4: ring-prefetched update / U passes (k_solve_pipe, k_solve_single): parity, then pipe A/B vs the round-3 form
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_r04h.log 2>&1 || { tail -30 gpurun_out/pytest_r04h.log; exit 1; }
tail -3 gpurun_out/pytest_r04h.log
timeout -k 10 400 python -u scripts/pipe_variants.py 0,5,4,1,2,0,5 > gpurun_out/pipe_ring_ab.jsonl 2>gpurun_out/pipe_ring_ab.err || { tail -20 gpurun_out/pipe_ring_ab.err; exit 1; }
cat gpurun_out/pipe_ring_ab.jsonl
