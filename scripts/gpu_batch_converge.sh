# Batched converge (F2) evidence on the GPU box: the per-phase breakdown and
# FETCH_SIZE / WRITE_SIZE passes (each its own rocprofv3 run) of k_solve_pipe
# (PIPE_OFF=1: k_solve_single) on infeasible and feasible iterates.  TAG names
# the outputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-bc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ -z "$NO_BREAKDOWN" ] && { timeout -k 10 300 python -u scripts/batch_converge_breakdown.py 1024 4096 4 ${VARIANTS:-fused_T,single_T,unfused_T,fused} > $OUT/breakdown.json 2> $OUT/breakdown.err || { tail -20 $OUT/breakdown.err; exit 1; }; cat $OUT/breakdown.json; }
[ -n "$NO_PMC" ] && exit 0
for F in "" 1; do
  sfx=${F:+_feasible}
  CASE=infeasible; [ -n "$F" ] && CASE=feasible
  FEASIBLE=$F timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$sfx -o kt -- python3 scripts/batch_converge_one.py 8 > $OUT/kt$sfx.log 2>&1 || { tail -20 $OUT/kt$sfx.log; exit 1; }
  FEASIBLE=$F timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch$sfx -o pmc -- python3 scripts/batch_converge_one.py 8 > $OUT/fetch$sfx.log 2>&1 || { tail -20 $OUT/fetch$sfx.log; exit 1; }
  FEASIBLE=$F timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write$sfx -o pmc -- python3 scripts/batch_converge_one.py 8 > $OUT/write$sfx.log 2>&1 || { tail -20 $OUT/write$sfx.log; exit 1; }
  echo "pmc$sfx done"
  python3 scripts/pmc_single.py $(ls $OUT/fetch$sfx/*counter_collection.csv) $(ls $OUT/write$sfx/*counter_collection.csv) $CASE ${PIPE_OFF:+single} || exit 1
done
