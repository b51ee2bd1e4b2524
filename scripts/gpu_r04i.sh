# Round 4: ring-prefetched passes, second box: pipe and k_solve_single A/B against the round-3 forms (variant 5), pipe PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/pipe_variants.py 0,5,0,5,0,5 > gpurun_out/pipe_ring_ab2.jsonl 2>gpurun_out/pipe_ring_ab2.err || { tail -20 gpurun_out/pipe_ring_ab2.err; exit 1; }
cat gpurun_out/pipe_ring_ab2.jsonl
PIPE_OFF=1 timeout -k 10 400 python -u scripts/pipe_variants.py 0,5,0,5 > gpurun_out/single_ring_ab.jsonl 2>gpurun_out/single_ring_ab.err || { tail -20 gpurun_out/single_ring_ab.err; exit 1; }
cat gpurun_out/single_ring_ab.jsonl
TAG=bc9 NO_BREAKDOWN=1 bash scripts/gpu_batch_converge.sh
