set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py tests/test_es_fft_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t/test.log 2>&1 || { tail -20 gpurun_out/t/test.log; exit 1; }
tail -1 gpurun_out/t/test.log
SDP_ES_SORT_PIECES=0 timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py -x -q --timeout 120 --timeout-method thread -k degrid > gpurun_out/t/test0.log 2>&1 || { tail -20 gpurun_out/t/test0.log; exit 1; }
tail -1 gpurun_out/t/test0.log
bash scripts/ab_env.sh gpurun_out/t/ab SDP_ES_SORT_PIECES "0 1" 2 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/t/kt.log 2>&1 || { tail -5 gpurun_out/t/kt.log; exit 1; }
find gpurun_out/t/kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/t/kernel_stats.csv \;
find gpurun_out/t/kt -name "*.csv" -delete
echo done
