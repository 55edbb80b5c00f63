#!/bin/bash
# Column-pass grid size A/B (SDP_ES_COL_ROUNDS: workgroups per CU slot).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--no-config3 --no-cpu-baseline --no-wstack --steps 10" scripts/kt_variants.sh gpurun_out/r4r \
    r2:ska-sdp-func_amd r1:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=1 r3:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=3 \
    r4:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=4 r8:ska-sdp-func_amd:SDP_ES_COL_ROUNDS=8 r2b:ska-sdp-func_amd || { echo kt failed; exit 1; }
find gpurun_out/r4r -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo call27 done
