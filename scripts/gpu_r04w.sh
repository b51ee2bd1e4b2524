# Round 4: k_solve_single held to 4 / 5 workgroups per CU (single_occ) on the horizon sweep (M = N/4) and the bench shape (pipe_off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/single_occ_ab.py > gpurun_out/single_occ_ab.jsonl 2>gpurun_out/single_occ_ab.err || { tail -20 gpurun_out/single_occ_ab.err; exit 1; }
cat gpurun_out/single_occ_ab.jsonl
