#!/bin/bash
cd "$GRAFT_REPO_ROOT"
scripts/herm_check.sh || exit $?
scripts/kt_top.sh gpurun_out/kt_h3 SDP_ES_HERM=1 || exit $?
scripts/pmc_traffic.sh gpurun_out/pmc_h3 --no-config3 --no-cpu-baseline --no-degrid --steps 2 --warmup 1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmc_h3 > gpurun_out/pmc_h3/summary.json; grep -A3 "herm\|k_rows\|k_cols" gpurun_out/pmc_h3/summary.json | head -40
