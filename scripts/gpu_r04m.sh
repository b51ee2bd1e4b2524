# Round 4: k_solve_mid2 builds held to 96 / 80 VGPRs (5 / 6 waves per SIMD) for workgroups of <= 6 waves (H = 2, 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
ARMS=def,lean5,lean6 timeout -k 10 300 python -u scripts/mid2_arms.py 2 3 > gpurun_out/mid2_lean.jsonl 2>gpurun_out/mid2_lean.err || { tail -20 gpurun_out/mid2_lean.err; exit 1; }
cat gpurun_out/mid2_lean.jsonl
