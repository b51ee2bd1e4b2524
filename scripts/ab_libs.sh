# A/B of library builds on the persistent fixed-mode launch (n_dual 1024,
# 1000 iterations): each lib named on the command line in turn, ROUNDS times,
# through scripts/persist_gate_ab.py (bits checked within each process).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    out=$(PQP_LIB=$lib timeout -k 10 100 python -u scripts/persist_gate_ab.py 0) || { echo "$lib failed"; exit 1; }
    med=$(echo "$out" | grep median | tr -d ' ,"' | cut -d: -f2)
    echo "$lib round $r: $med us/update"
  done
done
