# Round-5 check of the early-out gap tests: the solver tests, then the
# workloads whose decisions run per iterate (bundled converge, the MPC batch,
# the horizon leg, one n_dual 1024 converge solve)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-gap}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py tests/test_gpu_mid.py tests/test_gpu_converge.py tests/test_gpu_wave.py tests/test_gpu_pipe.py tests/test_gpu_batch_converge.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/bundled_timing.py 2>/dev/null | tail -1 | tee $O/bundled.json
timeout -k 10 120 python -u scripts/mpc_timing.py 2>/dev/null | tail -3 | tee $O/mpc.txt
for H in 2 3 4 5; do timeout -k 10 120 python -u scripts/horizon_pmc.py $H 2>/dev/null | tail -1; done | tee $O/horizon.txt
timeout -k 10 120 python -u scripts/converge_ab.py 2>/dev/null | tail -1 | tee $O/converge.json
