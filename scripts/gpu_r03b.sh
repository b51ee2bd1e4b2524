cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_batch_converge.py tests/test_gpu_parity.py tests/test_gpu_setup.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_b.log 2>&1 || { tail -40 gpurun_out/pt_b.log; exit 1; }
tail -3 gpurun_out/pt_b.log
timeout -k 10 300 python -u scripts/gj_timing.py 512 4096 > gpurun_out/gj.json 2>gpurun_out/gj.err || { tail gpurun_out/gj.err; exit 1; }
cat gpurun_out/gj.json
TAG=bc1 NO_PMC=1 bash scripts/gpu_batch_converge.sh
