set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/xcd
timeout -k 10 300 python -u -m pytest tests/test_es_gpu.py tests/test_es_fft_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xcd/test.log 2>&1 || { tail -20 gpurun_out/xcd/test.log; exit 1; }
tail -1 gpurun_out/xcd/test.log
bash scripts/ab_env.sh gpurun_out/xcd/ab SDP_ES_XCD_ORDER "0 1" 3 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
SDP_ES_XCD_ORDER=$v timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_bucket_fill --output-format csv -d gpurun_out/xcd/pmc$v/pass1 -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-degrid > gpurun_out/xcd/pmc$v.log 2>&1 || { echo pmc fail; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/xcd/pmc0 2>/dev/null | tail -8
python3 scripts/pmc_summary.py gpurun_out/xcd/pmc1 2>/dev/null | tail -8
echo done
