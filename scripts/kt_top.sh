#!/bin/bash
# Kernel-trace of the config-2 bench (gridding only) under the environment
# given as arguments; prints the per-kernel average durations (us).
#   scripts/kt_top.sh OUT [VAR=value ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --no-config3 --no-cpu-baseline --no-degrid --steps 5 > "$OUT/kt.log" 2>&1 || { tail -5 "$OUT/kt.log"; exit 1; }
f=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+(<[^>(]*>)?)", r["Name"])
    if m: print(f'{m.group(1)[:50]:50s} {float(r["AverageNs"])/1e3:9.1f} us x {r["Calls"]}')
PY
