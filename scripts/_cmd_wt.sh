set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wt3
timeout -k 10 400 python -u -m pytest tests/test_wstack_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wt3/test.log 2>&1 || { tail -30 gpurun_out/wt3/test.log; exit 1; }
tail -1 gpurun_out/wt3/test.log
for r in 1 2; do
timeout -k 10 300 python3 -u bench_wtower.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wt3/b_$r.json 2> gpurun_out/wt3/b_$r.err || { tail -5 gpurun_out/wt3/b_$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/wt3/b_$r.json
done
