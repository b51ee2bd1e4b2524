# SQ counters of k_solve_mid (scripts/mid_one.py), one rocprofv3 pass per set
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/mid_pmc; export TMPDIR=/tmp PYTHONUNBUFFERED=1
H=${H:-5}; B=${B:-4096}; MODE=${MODE:-fixed}; export MODE
rocprofv3 -L > gpurun_out/mid_pmc/avail.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/mid_pmc/p$i -o p$i -- python3 scripts/mid_one.py $H $B > gpurun_out/mid_pmc/p$i.log 2>&1 || { tail -5 gpurun_out/mid_pmc/p$i.log; exit 1; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mid_pmc/kt -o kt -- python3 scripts/mid_one.py $H $B > gpurun_out/mid_pmc/kt.log 2>&1 || { tail -5 gpurun_out/mid_pmc/kt.log; exit 1; }
echo done
