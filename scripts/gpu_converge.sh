# Persistent converge launch: parity tests then timings (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_converge.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_converge_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_converge_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_converge_$TAG.log
timeout -k 10 300 python -u scripts/converge_timing.py > gpurun_out/converge_timing_$TAG.txt 2>&1 || { tail -20 gpurun_out/converge_timing_$TAG.txt; exit 1; }
cat gpurun_out/converge_timing_$TAG.txt | grep n_dual
timeout -k 10 200 python -u scripts/converge_trace.py > gpurun_out/converge_trace_$TAG.json 2>&1 || { tail -20 gpurun_out/converge_trace_$TAG.json; exit 1; }
python - <<'PY' || true
import json, os
s = open(f"gpurun_out/converge_trace_{os.environ.get('TAG', 'c')}.json").read()
t = json.loads(s[s.index("{"):])
print({k: round(v, 2) for k, v in t["handover"].items()})
for k, v in t["timeline_from_decision_u-8"].items():
    print(k, v)
for k, v in t["roles"].items():
    if k.startswith("DEC") or ".w0" in k:
        print(k, {a: round(b, 2) for a, b in v.items()})
PY
