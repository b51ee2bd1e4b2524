# Round 4: k_solve_pipe's cost-phase sums interleaved and read 16 bytes at a time: parity and phase trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_r04s.log 2>&1 || { tail -30 gpurun_out/pytest_r04s.log; exit 1; }
tail -2 gpurun_out/pytest_r04s.log
timeout -k 10 300 python -u scripts/pipe_variants.py 0,0 > gpurun_out/pipe_costsums.jsonl 2>gpurun_out/pipe_costsums.err || { tail -20 gpurun_out/pipe_costsums.err; exit 1; }
cat gpurun_out/pipe_costsums.jsonl
timeout -k 10 300 python -u scripts/bc_leg.py > gpurun_out/bc_leg_costsums.json 2>gpurun_out/bc_leg_costsums.err || { tail -20 gpurun_out/bc_leg_costsums.err; exit 1; }
python -c "import json; b=json.load(open('gpurun_out/bc_leg_costsums.json')); [print(c, b[c]['ms_per_iteration_samples'], b[c]['frac_of_hbm_peak'], b[c]['ms_per_iteration_incl_launches']) for c in ('infeasible','feasible')]"
TAG=bc10 NO_BREAKDOWN=1 bash scripts/gpu_batch_converge.sh
