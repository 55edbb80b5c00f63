#!/bin/bash
# Config-4 A/B of library builds (scripts/variant_lib.sh): one kernel trace
# of bench_wtower (grid + degrid) per library dir, with the kernels whose
# names match REGEX listed. scripts/gpu_wt_lib_ab.sh OUT "dir_a dir_b" REGEX
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2; RE=${3:-k_}
mkdir -p "$OUT"
for d in $DIRS; do
    n=${d//\//_}
    ( export SKA_SDP_FUNC_LIB_DIR=$d; timeout -k 10 300 rocprofv3 --kernel-trace \
        --stats --output-format csv -d "$OUT/$n" -o kt -- python3 bench_wtower.py \
        --degrid --steps 1 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err" ) \
        || { tail -5 "$OUT/$n.err"; exit 1; }
    f=$(find "$OUT/$n" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/${n}_stats.csv" && find "$OUT/$n" -name "*.csv" ! -name "*kernel_stats.csv" -delete
    python3 - "$OUT/${n}_stats.csv" "$OUT/$n.json" "$d" "$RE" <<'PY'
import csv, json, re, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "grid", d["value"], "degrid", d["degrid"]["mvis_s"])
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[4], r["Name"]):
        print("   ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
echo ab done
