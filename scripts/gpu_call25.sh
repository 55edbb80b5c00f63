#!/bin/bash
# k_tower_dft block power from the pixel phase (SDP_DFT_TURNS): tower /
# w-stack parity, kernel-trace A/B against variants/turns0.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_wstack_gpu.py tests/test_wtower_gpu.py tests/test_wtower_vla_gpu.py -m gpu \
    > gpurun_out/r4t/tests.log 2>&1 || { tail -30 gpurun_out/r4t/tests.log; exit 1; }
tail -2 gpurun_out/r4t/tests.log
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4t/kt new:ska-sdp-func_amd base:variants/turns0 \
    new2:ska-sdp-func_amd base2:variants/turns0 || { echo kt failed; exit 1; }
timeout -k 10 300 python -u bench_wtower.py --degrid > gpurun_out/r4t/wtower.json 2> gpurun_out/r4t/wtower.err || { tail -5 gpurun_out/r4t/wtower.err; exit 1; }
tail -c 300 gpurun_out/r4t/wtower.json
find gpurun_out/r4t -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo call25 done
