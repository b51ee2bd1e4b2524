# Round 4: the N = 2 bench path rehearsed on one GPU over gloo with the final bench.py (self-launched ranks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
PQP_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --no-cpu-baseline > gpurun_out/bench_rehearse2_r04final.json 2> gpurun_out/bench_rehearse2_r04final.err || { tail -30 gpurun_out/bench_rehearse2_r04final.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_rehearse2_r04final.json')); print(d['n_gpus'], d['value'], d.get('gather_ok'), sorted(k for k in d if isinstance(d[k], dict)))"
