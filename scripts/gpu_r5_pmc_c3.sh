#!/bin/bash
# SQ counters of the config-3 tile kernel for two library builds.
#   scripts/gpu_r5_pmc_c3.sh OUT "libdir_a libdir_b"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2
for d in $DIRS; do
    f=${d//\//_}
    SKA_SDP_FUNC_LIB_DIR=$d timeout -k 10 400 scripts/pmc_sq.sh "$OUT/$f" "k_scatter_tab" \
        --rows 100000 --steps 1 --warmup 0 --no-degrid --no-wstack --c3-steps 1 --no-cpu-baseline || exit 1
    python3 scripts/pmc_summary.py "$OUT/$f" > "$OUT/$f.txt" 2>&1 || true
    cat "$OUT/$f.txt"
done
