# Round 4: the bench with the batch_converge leg warmed for 0.5 s
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r04p.json 2> gpurun_out/bench_r04p.err || { tail -30 gpurun_out/bench_r04p.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04p.json')); b=d['batch_converge']; print('bench', b['infeasible']['ms_per_iteration_samples'], b['infeasible']['frac_of_hbm_peak'], b['feasible']['ms_per_iteration_samples'], b['feasible']['frac_of_hbm_peak']); print(json.dumps(d['horizon'])[:400])"
