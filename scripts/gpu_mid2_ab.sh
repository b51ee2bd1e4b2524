# k_solve_mid2 A/B on the horizon workload (scripts/horizon_pmc.py): the
# library builds named on the command line (ab/libpqp_NAME.so) alternating,
# two rounds, H = 2..5.  Usage: bash scripts/gpu_mid2_ab.sh NAME...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/mid2_ab
for r in 1 2; do for H in ${HS:-2 3 4 5}; do for v in "$@"; do
  echo "$v H=$H $(PQP_LIB=ab/libpqp_$v.so timeout -k 10 120 python -u scripts/horizon_pmc.py $H 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["converge_ms"],2), "ms h_sum", d["h_sum"])')" || exit 1
done; done; done | tee gpurun_out/mid2_ab/ab.txt
