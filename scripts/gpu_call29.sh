#!/bin/bash
# Column-pass rounds A/B (SDP_ES_COL_ROUNDS) including the 3-D line's
# full-length column passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--no-config3 --no-cpu-baseline --steps 3 --warmup 1" scripts/kt_variants.sh gpurun_out/r4q \
    r2:ska-sdp-func_amd r3:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=3 r4:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=4 \
    r2b:ska-sdp-func_amd r3b:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=3 r4b:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=4 || { echo kt failed; exit 1; }
find gpurun_out/r4q -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo call29 done
