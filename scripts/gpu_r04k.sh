# Round 4: k_solve_pipe with whole-row Gp tiles (pipe_variant 6): parity, then A/B against the default tiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_r04k.log 2>&1 || { tail -30 gpurun_out/pytest_r04k.log; exit 1; }
tail -3 gpurun_out/pytest_r04k.log
timeout -k 10 400 python -u scripts/pipe_variants.py 0,6,0,6,0,6 > gpurun_out/pipe_rows_ab.jsonl 2>gpurun_out/pipe_rows_ab.err || { tail -20 gpurun_out/pipe_rows_ab.err; exit 1; }
cat gpurun_out/pipe_rows_ab.jsonl
