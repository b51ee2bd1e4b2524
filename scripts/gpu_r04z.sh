# Round 4: k_solve_single workgroups per CU chosen by shape and batch: parity and the horizon sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch_converge.py tests/test_gpu_pipe.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_r04z.log 2>&1 || { tail -30 gpurun_out/pytest_r04z.log; exit 1; }
tail -2 gpurun_out/pytest_r04z.log
timeout -k 10 400 python -u scripts/horizon_sweep.py 8 12 16 24 32 > gpurun_out/hsweep_occ2.jsonl 2>gpurun_out/hsweep_occ2.err || { tail -20 gpurun_out/hsweep_occ2.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/hsweep_occ2.jsonl'):
    d=json.loads(l); print(d['H'], d['n_dual'], d['batch'], round(d['batch_ms'],1), d['all_h_313'])"
