# k_solve_pipe variants: quick parity, then timing + phase traces per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-pv}
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python -u scripts/pipe_variants.py ${VARIANTS:-0,1,2,3} > gpurun_out/pv_$TAG.jsonl 2> gpurun_out/pv_$TAG.err || { tail -20 gpurun_out/pv_$TAG.err; exit 1; }
cat gpurun_out/pv_$TAG.jsonl
