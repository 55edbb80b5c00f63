#!/bin/bash
# Config-4 A/B: kernel traces of one gridding call (+ degrid) with and
# without an env switch. scripts/gpu_wt_ab.sh OUT VAR
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; VAR=$2
mkdir -p "$OUT"
run() {   # name, env prefix
    ( export "$2"; timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$OUT/$1" -o kt -- python3 bench_wtower.py \
        --degrid --steps 1 --no-cpu-baseline > "$OUT/$1.json" \
        2> "$OUT/$1.err" ) || { tail -5 "$OUT/$1.err"; return 1; }
    f=$(find "$OUT/$1" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/$1_stats.csv" && find "$OUT/$1" -name "*.csv" ! -name "*kernel_stats.csv" -delete
    tail -c 300 "$OUT/$1.json" | head -c 300; echo
}
run a "SDP_AB_NONE=1" || exit 1
run b "$VAR=1" || exit 1
echo ab done
