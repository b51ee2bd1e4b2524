# Round 4: k_solve_pipe with the CU's second workgroup started late (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/pipe_stagger_ab.py 0,300000,600000,1200000 > gpurun_out/pipe_stagger_r04f.jsonl 2>gpurun_out/pipe_stagger_r04f.err || { tail -20 gpurun_out/pipe_stagger_r04f.err; exit 1; }
cat gpurun_out/pipe_stagger_r04f.jsonl
