# Round 4 check: the whole GPU suite, smoke, mid2 arms, setup timing, and a
# default 1-GPU bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04e.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_r04e.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r04e.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04e.log 2>&1 || { tail -20 gpurun_out/smoke_r04e.log; exit 1; }
tail -1 gpurun_out/smoke_r04e.log
timeout -k 10 300 python -u scripts/mid2_arms.py 2 3 4 5 > gpurun_out/mid2_arms_r04e.jsonl 2>gpurun_out/mid2_arms_r04e.err || { tail -20 gpurun_out/mid2_arms_r04e.err; exit 1; }
cat gpurun_out/mid2_arms_r04e.jsonl
timeout -k 10 200 python -u scripts/setup_pk_timing.py 1024 512 64 3 > gpurun_out/setup_pk_r04e.json 2>gpurun_out/setup_pk_r04e.err || { tail -20 gpurun_out/setup_pk_r04e.err; exit 1; }
cat gpurun_out/setup_pk_r04e.json
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04e.json 2> gpurun_out/bench_r04e.err || { tail -30 gpurun_out/bench_r04e.err; exit 1; }
cat gpurun_out/bench_r04e.json
