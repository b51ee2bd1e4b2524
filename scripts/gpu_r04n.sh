# Round 4: k_solve_mid2's 80-VGPR build as the default for workgroups of <= 6 waves: parity (mid tests incl.
# the horizon populations) and arms at H = 2, 3 (default, the 128-VGPR build, lane sides, one lane per row)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mid.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_r04n.log 2>&1 || { tail -30 gpurun_out/pytest_r04n.log; exit 1; }
tail -3 gpurun_out/pytest_r04n.log
ARMS=def,fat,pair_lean,row_lean timeout -k 10 300 python -u scripts/mid2_arms.py 2 3 > gpurun_out/mid2_lean2.jsonl 2>gpurun_out/mid2_lean2.err || { tail -20 gpurun_out/mid2_lean2.err; exit 1; }
cat gpurun_out/mid2_lean2.jsonl
