# Round 4: k_solve_mid2 forms (one lane per row / lane sides) against
# k_solve_mid: parity (test_gpu_mid.py), A/B on the horizon sweep, phase trace;
# setup GEMM kernel stats; bundled fixed-1000 latency (k_fixed_tiny, DPP y_i)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_mid.py "tests/test_gpu_parity.py::test_bundled_fixed_1000_bit_exact" tests/test_gpu_parity.py::test_bundled_fixed_k_updates > gpurun_out/pt_r04c.log 2>&1 || { grep -E "PASSED|FAILED" gpurun_out/pt_r04c.log | tail -20; tail -60 gpurun_out/pt_r04c.log; exit 1; }
grep -E "passed|failed" gpurun_out/pt_r04c.log | tail -3
timeout -k 10 400 python -u scripts/mid2_ab.py 2 3 4 5 > gpurun_out/mid2_ab_r04c.jsonl 2>gpurun_out/mid2_ab_r04c.err || { tail -20 gpurun_out/mid2_ab_r04c.err; exit 1; }
cat gpurun_out/mid2_ab_r04c.jsonl
for pair in 0 1; do
B=4096 MODES=feasible MID2_PAIR=$pair timeout -k 10 200 python -u scripts/mid_trace.py 4 5 > gpurun_out/mid2_trace_r04c_p$pair.jsonl 2>&1 || { tail -20 gpurun_out/mid2_trace_r04c_p$pair.jsonl; exit 1; }
cat gpurun_out/mid2_trace_r04c_p$pair.jsonl
done
timeout -k 10 120 python -u scripts/bundled_timing.py > gpurun_out/bundled_r04c.json 2>&1 || { tail -20 gpurun_out/bundled_r04c.json; exit 1; }
cat gpurun_out/bundled_r04c.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/setup_pk_prof2 -o kt -- python3 -u scripts/setup_pk_timing.py 1024 512 64 1 > gpurun_out/setup_pk_prof2.log 2>&1 || { tail -20 gpurun_out/setup_pk_prof2.log; exit 1; }
find gpurun_out/setup_pk_prof2 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220 | head -20
