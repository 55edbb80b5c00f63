#!/bin/bash
# Round-4 A/B: correctness of the variants under test (short pytest
# subsets), then kernel traces of each (scripts/kt_variants.sh) with the
# per-kernel averages printed.  scripts/gpu_r4_ab.sh OUT "name:dir[:VAR=v] ..."
#   PRE: optional list of "dir:VAR=v:pytest-k" correctness runs ('+' in
#   the -k expression stands for a space).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; AB=$2
mkdir -p "$OUT"
for spec in $PRE; do
    IFS=: read -r d e k <<< "$spec"
    k=${k//+/ }                      # '+' stands for a space in -k
    env SKA_SDP_FUNC_LIB_DIR="$d" $e timeout -k 10 300 python -u -m pytest \
        tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$k" \
        > "$OUT/pre_$(basename "$d").log" 2>&1 \
        || { echo "FAILED: $spec"; tail -30 "$OUT/pre_$(basename "$d").log"; exit 1; }
    echo "ok $spec: $(tail -1 "$OUT/pre_$(basename "$d").log")"
done
scripts/kt_variants.sh "$OUT/ab" $AB || exit 1
for spec in $AB; do
    n=${spec%%:*}
    f=$(find "$OUT/ab/$n" -name "*kernel_stats.csv" | head -1)
    echo "== $n"
    python3 - "$f" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+(<[^>(]*>)?)", r["Name"])
    if m and float(r["AverageNs"]) > 20e3:
        print(f'{m.group(1)[:50]:50s} {float(r["AverageNs"])/1e3:9.1f} us x {r["Calls"]}')
PY
done
