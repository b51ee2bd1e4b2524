# timelines of the persistent fixed-mode launch (split form, then the one-XCD lean
# form) and the lean A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06g}
timeout -k 10 120 python scripts/persist_trace.py > gpurun_out/persist_trace_split_$T.json 2>&1 && LEAN=1 timeout -k 10 120 python scripts/persist_trace.py > gpurun_out/persist_trace_lean_$T.json 2>&1 && timeout -k 10 120 python scripts/persist_lean_ab.py 5 > gpurun_out/persist_lean_ab_$T.json 2> gpurun_out/persist_lean_ab_$T.err
rc=$?
T=$T python3 - <<'PY'
import json,os
T=os.environ["T"]
for f in ("split","lean"):
    try:
        s=open(f"gpurun_out/persist_trace_{f}_{T}.json").read(); d=json.loads(s[s.index("{"):])
        print(f, d["us_per_update_untraced"], d["clocks_per_update"], {w: v["adds (turn -> chain done)"] for w,v in d["per_wave_median_clocks"].items()}, d["exchange_clocks (last wave done u -> wave 0 staged u+1)"], d["handoff_clocks_per_pair"])
    except Exception as e: print(f, "err", e)
PY
cat gpurun_out/persist_lean_ab_$T.json
exit $rc
