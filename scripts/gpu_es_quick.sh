#!/bin/bash
# ES quick check: the ES GPU tests, then a config-2 kernel trace summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/esq}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_es_gpu.py tests/test_es_batches_gpu.py tests/test_es_fft_gpu.py \
    tests/test_es_multichan_gpu.py tests/test_distributed_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/kt" -o kt -- python3 bench.py --steps 20 --warmup 3 \
    --no-cpu-baseline --no-config3 --no-wstack > "$OUT/bench.json" \
    2> "$OUT/kt.log" || { tail -5 "$OUT/kt.log"; exit 1; }
f=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/stats.csv" && find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
python3 - "$OUT/stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:18]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
echo esq done
