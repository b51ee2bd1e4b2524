# Round check on the GPU box: GPU suite, smoke, the self-launched 2-rank
# rehearsal and a 1-GPU bench line.  TAG names the outputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
if [ -z "$SKIP_REHEARSE" ]; then
PQP_BENCH_REHEARSE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --rowshard-updates 20 > gpurun_out/bench_rehearse2_$TAG.json 2> gpurun_out/bench_rehearse2_$TAG.err || { tail -30 gpurun_out/bench_rehearse2_$TAG.err; exit 1; }
cat gpurun_out/bench_rehearse2_$TAG.json
# the same with rank 1's row block failing inside the leg: the line must survive (rc 0)
PQP_BENCH_REHEARSE=1 PQP_BENCH_FAULT=rowshard:1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --rowshard-updates 20 > gpurun_out/bench_rehearse2_fault_$TAG.json 2> gpurun_out/bench_rehearse2_fault_$TAG.err || { tail -30 gpurun_out/bench_rehearse2_fault_$TAG.err; exit 1; }
cat gpurun_out/bench_rehearse2_fault_$TAG.json
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
