# Round 4 check: the whole GPU suite, smoke, a default 1-GPU bench line, and
# the round's rocprofv3 evidence (kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04final.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_r04final.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r04final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04final.log 2>&1 || { tail -20 gpurun_out/smoke_r04final.log; exit 1; }
tail -1 gpurun_out/smoke_r04final.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04final.json 2> gpurun_out/bench_r04final.err || { tail -30 gpurun_out/bench_r04final.err; exit 1; }
cat gpurun_out/bench_r04final.json
