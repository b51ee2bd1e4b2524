# A/B of library builds on the persistent converge launch (n_dual 1024, cap
# 2000): each lib named on the command line in turn, ROUNDS times, through
# scripts/converge_ab.py (digest of Y*, U* printed for a bit-for-bit check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    out=$(PQP_LIB=$lib timeout -k 10 100 python -u scripts/converge_ab.py) || { echo "$lib failed"; exit 1; }
    echo "$lib round $r: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["median_us_per_iter"],3), "us/iter (slope", round(d["slope_us_per_iter"],3), "fixed", round(d["per_solve_fixed_us"],1), "us) digest", d["digest"], "h", d["h"])')"
  done
done
