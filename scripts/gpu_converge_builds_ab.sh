# configs[2] converge-mode builds, two rounds, each build in its own process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/converge_builds_ab_${TAG:-r06l}.jsonl
: > $O
for r in 1 2; do
  for v in ${VARIANTS:-c0 t1 t2 t8 n2 n8}; do
    PQP_LIB=ab/libpqp_$v.so timeout -k 10 90 python scripts/converge_build_time.py $v >> $O 2>/dev/null || exit 1
  done
done
cat $O
