# k_solve_pipe 128 x 96 single-slot tiles (pipe_variant 3) vs 64 x 64 (0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_big.log 2>&1 || { tail -40 gpurun_out/pt_big.log; exit 1; }
tail -1 gpurun_out/pt_big.log
timeout -k 10 300 python -u scripts/pipe_variants.py 0,3,0,3 > gpurun_out/pv_big.jsonl 2> gpurun_out/pv_big.err || { tail -20 gpurun_out/pv_big.err; exit 1; }
cat gpurun_out/pv_big.jsonl
