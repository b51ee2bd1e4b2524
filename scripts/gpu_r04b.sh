# Round 4: the rest of the first call's list (setup / batch-converge / pipe /
# population / shard tests), timings (setup GEMM, mid2 vs mid, mid2 trace),
# then configs[4] rehearsed at its real size on one GPU (8 ranks x 4096
# problems of n_dual 1024 over gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_setup.py tests/test_gpu_batch_converge.py tests/test_gpu_pipe.py::test_pipe_bench_size_infeasible_vs_oracle \
  "tests/test_gpu_parity.py::test_mpc_population_vs_reference" "tests/test_gpu_parity.py::test_mpc_batch_of_states_vs_oracle" \
  tests/test_gpu_shard.py > gpurun_out/pt_r04b.log 2>&1 || { grep -E "PASSED|FAILED" gpurun_out/pt_r04b.log | tail -20; tail -60 gpurun_out/pt_r04b.log; exit 1; }
grep -E "passed|failed" gpurun_out/pt_r04b.log | tail -3
timeout -k 10 300 python -u scripts/mid2_ab.py 2 3 4 5 > gpurun_out/mid2_ab_r04b.jsonl 2>gpurun_out/mid2_ab_r04b.err || { tail -20 gpurun_out/mid2_ab_r04b.err; exit 1; }
cat gpurun_out/mid2_ab_r04b.jsonl
B=4096 MODES=feasible timeout -k 10 200 python -u scripts/mid_trace.py 4 > gpurun_out/mid2_trace_r04b.jsonl 2>&1 || { tail -20 gpurun_out/mid2_trace_r04b.jsonl; exit 1; }
cat gpurun_out/mid2_trace_r04b.jsonl
timeout -k 10 200 python -u scripts/setup_pk_timing.py 1024 512 64 3 > gpurun_out/setup_pk_r04b.json 2>gpurun_out/setup_pk_r04b.err || { tail -20 gpurun_out/setup_pk_r04b.err; exit 1; }
cat gpurun_out/setup_pk_r04b.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/setup_pk_prof -o kt -- python3 -u scripts/setup_pk_timing.py 1024 512 64 1 > gpurun_out/setup_pk_prof.log 2>&1 || { tail -20 gpurun_out/setup_pk_prof.log; exit 1; }
find gpurun_out/setup_pk_prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -20
PQP_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 8 --batch 4096 --steps 20 --warmup 2 --no-cpu-baseline \
  --rowshard-updates 20 > gpurun_out/bench_rehearse8_r04b.json 2> gpurun_out/bench_rehearse8_r04b.err || { tail -40 gpurun_out/bench_rehearse8_r04b.err; exit 1; }
cat gpurun_out/bench_rehearse8_r04b.json
