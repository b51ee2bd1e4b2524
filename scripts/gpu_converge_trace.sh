cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/converge_trace.py > gpurun_out/converge_trace_c4.json 2>&1
