# Round 4: k_solve_single's cost sums interleaved: parity, and the horizon sweep (M = N/4: k_solve_single) before/after, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_converge.py tests/test_gpu_pipe.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_r04u.log 2>&1 || { tail -30 gpurun_out/pytest_r04u.log; exit 1; }
tail -2 gpurun_out/pytest_r04u.log
for r in 1 2; do
  PQP_LIB=$GRAFT_REPO_ROOT/pqp-for-mpc_amd/pqp_amd/libpqp_before.so timeout -k 10 300 python -u scripts/horizon_sweep.py 8 16 32 > gpurun_out/hsweep_before_$r.jsonl 2>gpurun_out/hsweep_before_$r.err || { tail -20 gpurun_out/hsweep_before_$r.err; exit 1; }
  timeout -k 10 300 python -u scripts/horizon_sweep.py 8 16 32 > gpurun_out/hsweep_after_$r.jsonl 2>gpurun_out/hsweep_after_$r.err || { tail -20 gpurun_out/hsweep_after_$r.err; exit 1; }
done
for f in gpurun_out/hsweep_*.jsonl; do echo $f; cut -c1-300 $f; done
TAG=bc11 NO_BREAKDOWN=1 bash scripts/gpu_batch_converge.sh
