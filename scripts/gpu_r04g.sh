# Round 4: horizon-problem tests (incl. the problem the reference never stops) and packed-GJ timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_mid.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_mid_r04g.log 2>&1 || { tail -30 gpurun_out/pytest_mid_r04g.log; exit 1; }
tail -3 gpurun_out/pytest_mid_r04g.log
timeout -k 10 200 python -u scripts/gj_timing.py 512 4096 > gpurun_out/gj_timing_r04g.json 2>gpurun_out/gj_timing_r04g.err || { tail -20 gpurun_out/gj_timing_r04g.err; exit 1; }
cat gpurun_out/gj_timing_r04g.json
