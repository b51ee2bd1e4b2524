# Round 4: k_solve_mid2 arms (C rows per wave, update-wave priority, pair form)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_mid.py > gpurun_out/pt_r04d.log 2>&1 || { tail -60 gpurun_out/pt_r04d.log; exit 1; }
tail -1 gpurun_out/pt_r04d.log
timeout -k 10 500 python -u scripts/mid2_arms.py 2 3 4 5 > gpurun_out/mid2_arms_r04d.jsonl 2>gpurun_out/mid2_arms_r04d.err || { tail -20 gpurun_out/mid2_arms_r04d.err; exit 1; }
cat gpurun_out/mid2_arms_r04d.jsonl
B=4096 MODES=feasible timeout -k 10 200 python -u scripts/mid_trace.py 4 5 > gpurun_out/mid2_trace_r04d.jsonl 2>&1 || { tail -20 gpurun_out/mid2_trace_r04d.jsonl; exit 1; }
cat gpurun_out/mid2_trace_r04d.jsonl
