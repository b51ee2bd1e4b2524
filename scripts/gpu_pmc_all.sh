# Every PMC record the bench line reads, for the current kernel sources:
# headline kernel trace + FETCH / WRITE passes, k_solve_pipe passes (F2), and
# k_solve_mid2 VALU passes (horizon); each step under its own limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r06fin}
bash scripts/gpu_profile.sh $T "--steps 20 --warmup 5 --no-cpu-baseline --no-bundled --rowshard-n 0" &&
NO_BREAKDOWN=1 TAG=bc_$T bash scripts/gpu_batch_converge.sh &&
bash scripts/gpu_r06.sh hpmc hpmc_$T
