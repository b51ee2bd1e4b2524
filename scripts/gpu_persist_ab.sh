# Persistent launches: parity tests, then fixed-mode and converge-mode timings (GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_converge.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/persist_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/persist_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/persist_tests_$TAG.log
timeout -k 10 200 python -u scripts/single_timing.py > gpurun_out/single_timing_$TAG.json 2>&1 || exit 1
timeout -k 10 200 python -u scripts/persist_trace.py > gpurun_out/persist_trace_$TAG.json 2>&1 || exit 1
timeout -k 10 300 python -u scripts/converge_timing.py 1024 > gpurun_out/converge_timing_$TAG.txt 2>&1 || exit 1
python - <<'PY'
import json, os
tag = os.environ.get("TAG", "p")
def load(f):
    s = open(f).read(); return json.loads(s[s.index("{"):])
st = load(f"gpurun_out/single_timing_{tag}.json")
print("single persistent us/update:", st["persistent"]["us_per_iter"], "bit_identical:", st["bit_identical"])
pt = load(f"gpurun_out/persist_trace_{tag}.json")
print({k: v for k, v in pt.items() if "clocks" in k or "us_per" in k})
for line in open(f"gpurun_out/converge_timing_{tag}.txt"):
    if line.startswith("{") and "n_dual" in line:
        d = json.loads(line); print("converge", d["n_dual"], d.get("persistent_cap2000"), d.get("bit_identical"))
PY
