# k_solve_mid forms: parity tests, per-phase trace and the horizon sweep with
# the stored-split form on (MID_SPLIT=1) and off (0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_gpu_mid.py tests/test_gpu_parity.py tests/test_gpu_batch_converge.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_mid.log 2>&1 || { tail -30 gpurun_out/pt_mid.log; exit 1; }
tail -1 gpurun_out/pt_mid.log
for sp in 0 1; do
  MID_SPLIT=$sp timeout -k 10 200 python -u scripts/mid_trace.py 2 3 4 5 > gpurun_out/mid_trace_s$sp.jsonl 2>gpurun_out/mid_trace.err || exit 1
  MID_SPLIT=$sp timeout -k 10 300 python -u scripts/horizon_sweep.py 2 3 4 5 > gpurun_out/horizon_s$sp.jsonl 2>gpurun_out/horizon.err || exit 1
done
python3 - <<'PY'
import json
for sp in (0, 1):
    for l in open(f"gpurun_out/horizon_s{sp}.jsonl"):
        d = json.loads(l)
        print("split" if sp == 1 else "qd   ", d["H"], d["n_dual"], "path", d["batch_path"], "ms %.2f" % d["batch_ms"], "solves/s %.0f" % d["qp_solves_per_s"], "off_ms", d.get("mid_off_batch_ms"), d.get("mid_off_same_bits"))
PY
