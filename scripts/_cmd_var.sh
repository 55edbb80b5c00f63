set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for r in 1 2; do
for v in var_c var_a var_b; do
  SKA_SDP_FUNC_LIB_DIR=$GRAFT_REPO_ROOT/$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/var/$v.$r.json 2> gpurun_out/var/$v.$r.err || { tail -5 gpurun_out/var/$v.$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['phases_ms']['tile_kernel'], d['degrid']['mvis_s'], d['degrid']['phases_ms'])" gpurun_out/var/$v.$r.json $v
done
done
SKA_SDP_FUNC_LIB_DIR=$GRAFT_REPO_ROOT/var_a timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var/test_a.log 2>&1 || { tail -20 gpurun_out/var/test_a.log; exit 1; }
tail -1 gpurun_out/var/test_a.log
SKA_SDP_FUNC_LIB_DIR=$GRAFT_REPO_ROOT/var_b timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var/test_b.log 2>&1 || { tail -20 gpurun_out/var/test_b.log; exit 1; }
tail -1 gpurun_out/var/test_b.log
