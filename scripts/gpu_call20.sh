#!/bin/bash
# Lagged-layer k_tower_dft A/B (SDP_DFT_LAG=1 at 4 and 3 waves per SIMD).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4o
for v in lag4 lag3; do
  SKA_SDP_FUNC_LIB_DIR=variants/$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wstack or wtower" > gpurun_out/r4o/pre_$v.log 2>&1 || { tail -20 gpurun_out/r4o/pre_$v.log; exit 1; }
  tail -1 gpurun_out/r4o/pre_$v.log
done
BENCH=bench_wtower.py BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4o/ab new:ska-sdp-func_amd lag4:variants/lag4 lag3:variants/lag3 new2:ska-sdp-func_amd || exit 1
python3 scripts/ab_table.py gpurun_out/r4o new lag4 lag3 new2 --top 6
