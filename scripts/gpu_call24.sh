#!/bin/bash
# k_tower_idft swizzled tap rows: tower/w-stack parity, kernel-trace A/B
# against the padded-row build (variants/swz0), LDS conflict counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4s
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_wstack_gpu.py tests/test_wtower_gpu.py tests/test_wtower_vla_gpu.py -m gpu \
    > gpurun_out/r4s/tests.log 2>&1 || { tail -30 gpurun_out/r4s/tests.log; exit 1; }
tail -2 gpurun_out/r4s/tests.log
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4s/kt swz:ska-sdp-func_amd base:variants/swz0 \
    swz2:ska-sdp-func_amd base2:variants/swz0 || { echo kt failed; exit 1; }
for v in ska-sdp-func_amd variants/swz0; do
  n=$(basename $v)
  SKA_SDP_FUNC_LIB_DIR=$v timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex "k_tower_idft" --output-format csv -d gpurun_out/r4s/pmc_$n -o pmc -- python3 bench_wtower.py --degrid --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4s/pmc_$n.log 2>&1 || { echo "$n pmc failed"; tail -3 gpurun_out/r4s/pmc_$n.log; exit 1; }
done
find gpurun_out/r4s -name "*.csv" ! -name "*kernel_stats.csv" ! -name "*counter_collection.csv" -delete
echo call24 done
