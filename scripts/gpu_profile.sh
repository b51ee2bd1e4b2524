# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun).
#   1) kernel trace + stats of a short bench run (per-kernel durations)
#   2) two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic
# Each step has its own time limit; any failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS=${2:---steps 20 --warmup 3 --no-cpu-baseline --no-bundled}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS > $OUT/kt_bench.json 2> $OUT/kt.err || exit $?
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py $ARGS > $OUT/pmc_fetch_bench.json 2> $OUT/pmc_fetch.err || exit $?
echo "fetch pass done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py $ARGS > $OUT/pmc_write_bench.json 2> $OUT/pmc_write.err || exit $?
echo "write pass done"
find $OUT -name "*.csv" | head -20
