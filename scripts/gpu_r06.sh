# GPU steps, one script: bash scripts/gpu_r06.sh STEP [TAG] (rounds 5-6)
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
tiny)
  # configs[1] on k_fixed_one / k_solve_quintet: parity first, then the A/B timing
  # and its kernel durations
  timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_handles.py tests/test_gpu_converge.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] &&
  timeout -k 10 180 python -u scripts/bundled_timing.py > $O/ab.json 2>&1 && cat $O/ab.json &&
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 -u scripts/bundled_timing.py 50 1 > $O/prof.log 2>&1 && tail -2 $O/prof.log
  ;;
trio)
  timeout -k 10 120 python -u scripts/trio_trace.py > $O/trio.json 2>&1; cat $O/trio.json
  ;;
iterab)
  timeout -k 10 300 python -u scripts/iterate_ab.py > $O/iterate_ab.json 2>&1; cat $O/iterate_ab.json
  ;;
headline)
  # the batched iterate's parity, then its rocprofv3 kernel trace and the
  # FETCH_SIZE / WRITE_SIZE passes behind profiles/pmc_traffic.json
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] &&
  bash scripts/gpu_profile.sh $TAG && cat gpurun_out/prof_$TAG/kt_bench.json
  # (then, here: python scripts/pmc_traffic.py gpurun_out/prof_TAG/pmc_fetch/..csv ..pmc_write/..csv 1024 4096 10)
  ;;
pytest)
  # bash scripts/gpu_r05.sh pytest TAG <pytest args...>
  shift 2
  timeout -k 10 900 python -u -m pytest "$@" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; exit $rc
  ;;
hpmc)
  # k_solve_mid2's VALU counters on the bench's horizon workload, H = 2, 4, 5:
  # one rocprofv3 pass per H (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES,
  # GRBM_GUI_ACTIVE) beside a kernel trace of the same command
  # (and the dense companion d112 / d140 of bench.py's horizon_dense leg)
  for H in 2 4 5 d112 d140; do
    D=$O/h$H; case $H in d*) D=$O/$H;; esac
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $D -o pmc -- python3 scripts/horizon_pmc.py $H > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
    cat $D.json
  done
  ;;
hlds)
  # k_solve_mid2's wave-state and LDS counters (where the phase's cycles go):
  # one pass per workload, SQ only (8 counters)
  for H in ${HLDS_SET:-4 5 d140}; do
    D=$O/l$H
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $D -o pmc -- python3 scripts/horizon_pmc.py $H > $D.json 2> $D.err || { tail -5 $D.err; exit 1; }
    cat $D.json
  done
  ;;
hab)
  # horizon A/B: bash scripts/gpu_r05.sh hab TAG "H knob=v ..." "H knob=v ..." ...
  shift 2
  for args in "$@"; do
    timeout -k 10 120 python -u scripts/horizon_pmc.py $args || exit 1
  done
  ;;
gj)
  # Gauss_Jordan: parity of every form (incl. non-finite inputs), then the timing
  timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -k gauss_jordan -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] &&
  timeout -k 10 300 python -u scripts/gj_timing.py 512 4096 > $O/gj_timing.json 2>&1 && cat $O/gj_timing.json &&
  timeout -k 10 300 python -u scripts/gj_timing.py 256 4096 > $O/gj_timing_256.json 2>&1 && cat $O/gj_timing_256.json
  ;;
bcab)
  # batch_converge (F2) on the round-4, round-5 and current libraries, same box,
  # alternating (is 0.848 / 0.853 box variance or a
  # regression?).  ab/r04 and ab/r05 hold each round's bench.py, bc_leg.py and
  # built pqp_amd (made here from git worktrees of 50a0bfe / a31e5a0)
  for r in 1 2; do
    for t in ab/r04 ab/r05 .; do
      l=$(basename $t); [ "$l" = . ] && l=r06
      timeout -k 10 240 python -u $t/scripts/bc_leg.py > $O/bc_${l}_$r.json 2> $O/bc_${l}_$r.err || { tail -5 $O/bc_${l}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], [(c, round(d[c]['ms_per_iteration'],3), round(d[c]['frac_of_hbm_peak'],4)) for c in ('infeasible','feasible')])" $O/bc_${l}_$r.json $l $r
    done
  done
  ;;
doorbell)
  timeout -k 10 120 ./scripts/probes/doorbell_probe 2000 > $O/doorbell.json 2>&1; rc=$?; cat $O/doorbell.json; exit $rc
  ;;
*)
  echo "unknown step $STEP"; exit 2;;
esac
