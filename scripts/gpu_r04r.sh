# Round 4: the batch_converge leg measured within one launch and with launches amortized
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/bc_leg.py > gpurun_out/bc_leg.json 2>gpurun_out/bc_leg.err || { tail -20 gpurun_out/bc_leg.err; exit 1; }
python -c "import json; b=json.load(open('gpurun_out/bc_leg.json')); [print(c, b[c]['ms_per_iteration_samples'], b[c]['frac_of_hbm_peak'], b[c]['ms_per_iteration_incl_launches'], b[c]['frac_of_hbm_peak_incl_launches'], b[c].get('k_solve_single_ms_per_iteration')) for c in ('infeasible','feasible')]"
