set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wt
timeout -k 10 400 python -u -m pytest tests/test_wstack_gpu.py tests/test_wtower_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wt/test.log 2>&1 || { tail -30 gpurun_out/wt/test.log; exit 1; }
tail -1 gpurun_out/wt/test.log
for v in rocfft fused; do
  SDP_WT_FFT=$v timeout -k 10 300 python3 -u bench_wtower.py --steps 2 --warmup 1 --degrid --no-cpu-baseline > gpurun_out/wt/b_$v.json 2> gpurun_out/wt/b_$v.err || { tail -5 gpurun_out/wt/b_$v.err; exit 1; }
  tail -1 gpurun_out/wt/b_$v.json | cut -c1-200
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['degrid']['mvis_s'], d['degrid']['ms_per_step'])" gpurun_out/wt/b_$v.json $v
done
