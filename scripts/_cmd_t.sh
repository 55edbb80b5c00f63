set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py tests/test_es_fft_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t/test.log 2>&1 || { tail -20 gpurun_out/t/test.log; exit 1; }
tail -1 gpurun_out/t/test.log
bash scripts/ab_env.sh gpurun_out/t/ab SDP_ES_COL_ROUNDS "1 2 3" 2 || exit $?
echo done
