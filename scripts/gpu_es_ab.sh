#!/bin/bash
# Config-2 A/B of an env switch: bench.py line + kernel trace per side.
#   scripts/gpu_es_ab.sh OUT VAR [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; VAR=$2; shift 2
mkdir -p "$OUT"
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-wstack $*"
run() {   # name, assignment
    ( export "$2"; timeout -k 10 300 python3 -u bench.py $ARGS > "$OUT/$1.json" \
        2> "$OUT/$1.err" ) || { tail -5 "$OUT/$1.err"; return 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'], d['phases_ms'], (d.get('degrid') or {}).get('mvis_s'))"
    ( export "$2"; timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$OUT/$1kt" -o kt -- python3 bench.py $ARGS \
        > "$OUT/$1kt.log" 2>&1 ) || { tail -5 "$OUT/$1kt.log"; return 1; }
    f=$(find "$OUT/$1kt" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/$1_stats.csv" && find "$OUT/$1kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
    python3 - "$OUT/$1_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("   ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
}
run a "SDP_AB_NONE=1" && run b "$VAR=1" && run a2 "SDP_AB_NONE=1" && echo ab done
