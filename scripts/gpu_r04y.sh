# Round 4: k_solve_single workgroups per CU (3 / 4 / 5) at the horizon sweep's other sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
HS=12,24,32 timeout -k 10 500 python -u scripts/single_occ_ab.py > gpurun_out/single_occ_ab2.jsonl 2>gpurun_out/single_occ_ab2.err || { tail -20 gpurun_out/single_occ_ab2.err; exit 1; }
cat gpurun_out/single_occ_ab2.jsonl
