#!/bin/bash
# Round 5: kernel trace of the config-3 gridding call (10 M rows x 64
# channels on one GPU), config 2 shrunk to a token size.
#   scripts/gpu_r5_c3.sh OUT
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r5c3}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/kt" -o kt -- python3 bench.py --rows 100000 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-degrid --no-wstack --c3-steps 2 > "$OUT/kt.log" 2>&1 \
    || { tail -5 "$OUT/kt.log"; exit 1; }
f=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+(<[^>(]*>)?)", r["Name"])
    if m: print(f'{m.group(1)[:60]:60s} {float(r["AverageNs"])/1e3:9.1f} us x {r["Calls"]}  tot {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
tail -c 1500 "$OUT/kt.log"
