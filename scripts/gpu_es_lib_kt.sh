#!/bin/bash
# Config-2 kernel traces of library builds (scripts/variant_lib.sh), one per
# dir, listing the kernels whose names match REGEX (average us):
#   scripts/gpu_es_lib_kt.sh OUT "dir_a dir_b" REGEX [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2; RE=${3:-k_}; shift 3
mkdir -p "$OUT"
i=0
for d in $DIRS; do
    i=$((i+1)); n=v$i
    ( export SKA_SDP_FUNC_LIB_DIR=$d; timeout -k 10 300 rocprofv3 --kernel-trace \
        --stats --output-format csv -d "$OUT/$n" -o kt -- python3 bench.py \
        --steps 20 --warmup 3 --no-cpu-baseline --no-wstack "$@" > "$OUT/$n.json" \
        2> "$OUT/$n.err" ) || { tail -5 "$OUT/$n.err"; exit 1; }
    f=$(find "$OUT/$n" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/${n}_stats.csv" && find "$OUT/$n" -name "*.csv" ! -name "*kernel_stats.csv" -delete
    python3 - "$OUT/${n}_stats.csv" "$d" "$RE" <<'PY'
import csv, re, sys
print(sys.argv[2])
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", r["Name"])
        print("   %-58s %5s %9.1f us" % (m.group(1) if m else r["Name"][:58],
              r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
echo kt done
