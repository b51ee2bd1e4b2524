# Default bench line + rocprofv3 kernel stats over every bench leg (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-v9}
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo "bench done"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_all_$TAG -o kt -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_all_$TAG.json 2> gpurun_out/prof_all_$TAG.err || { tail -20 gpurun_out/prof_all_$TAG.err; exit 1; }
echo "rocprof done"
find gpurun_out/prof_all_$TAG -name "*stats.csv"
