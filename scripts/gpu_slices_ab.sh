# configs[2] slice-size builds, two rounds, each build in its own process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/slices_ab_${TAG:-r06h}.jsonl
: > $O
for r in 1 2; do
  for v in ${VARIANTS:-s24a s20 s28 s24b s16}; do
    PQP_LIB=ab/libpqp_$v.so timeout -k 10 60 python scripts/persist_slice_time.py $v >> $O 2>/dev/null || exit 1
  done
done
cat $O
