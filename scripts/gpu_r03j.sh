# k_solve_pipe: parity tests, then the batched converge breakdown (pipe vs
# k_solve_single) at n_dual 1024 x 4096
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-pipe}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python -u scripts/batch_converge_breakdown.py 1024 4096 4 ${VARIANTS:-fused_T,single_T} > gpurun_out/bd_$TAG.json 2> gpurun_out/bd_$TAG.err || { tail -20 gpurun_out/bd_$TAG.err; exit 1; }
cat gpurun_out/bd_$TAG.json
timeout -k 10 200 python -u scripts/pipe_trace.py 8 > gpurun_out/trace_$TAG.jsonl 2> gpurun_out/trace_$TAG.err || { tail -20 gpurun_out/trace_$TAG.err; exit 1; }
cat gpurun_out/trace_$TAG.jsonl
