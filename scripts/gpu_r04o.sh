# Round 4: the batch_converge leg in the bench vs standalone on the same box: before the bench, the bench itself, after it
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/pipe_variants.py 0,0 > gpurun_out/pipe_before.jsonl 2>gpurun_out/pipe_before.err || { tail -20 gpurun_out/pipe_before.err; exit 1; }
cat gpurun_out/pipe_before.jsonl
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r04o.json 2> gpurun_out/bench_r04o.err || { tail -30 gpurun_out/bench_r04o.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04o.json')); b=d['batch_converge']; print('bench', b['infeasible']['ms_per_iteration_samples'], b['feasible']['ms_per_iteration_samples'])"
timeout -k 10 200 python -u scripts/pipe_variants.py 0,0 > gpurun_out/pipe_after.jsonl 2>gpurun_out/pipe_after.err || { tail -20 gpurun_out/pipe_after.err; exit 1; }
cat gpurun_out/pipe_after.jsonl
