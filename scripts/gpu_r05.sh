# Round 5 GPU steps, one script: bash scripts/gpu_r05.sh STEP [TAG]
# Every GPU step runs under its own time limit and the steps are chained
# with &&, so a fault or a timeout ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
STEP=$1
TAG=${2:-$1}
O=gpurun_out/$TAG
mkdir -p $O
case $STEP in
bundled)
  # configs[1]: wall time per pqp_problem_solve, the kernel durations under
  # rocprofv3, and the fixed-mode forms of scripts/probes/bundled_probe.hip
  timeout -k 10 120 python -u scripts/bundled_timing.py > $O/wall.json 2>&1 && cat $O/wall.json &&
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 -u scripts/bundled_timing.py > $O/prof.log 2>&1 && tail -3 $O/prof.log &&
  python scripts/probes/bundled_probe_data.py $O/bundled.bin &&
  timeout -k 10 60 ./scripts/probes/bundled_probe $O/bundled.bin 200 > $O/probe.jsonl 2>&1; cat $O/probe.jsonl
  ;;
*)
  echo "unknown step $STEP"; exit 2;;
esac
