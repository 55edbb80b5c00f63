#!/bin/bash
# Round-4 GPU check: the ES parity tests touched by a change (2-D / 3-D,
# fused FFT, batches, the 3-D config-2-geometry oracle test), the bench
# line, and a kernel trace of the bench without config 3 / CPU baselines.
#   scripts/gpu_r4_check.sh OUT [pytest -k expression]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r4}
K=${2:-"test_es_gpu or test_es_fft_gpu or batches or wstacking"}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 \
    --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('grid', d['value'], d['phases_ms']); print('degrid', round(d['degrid']['mvis_s'],1), d['degrid']['phases_ms'])
print('c3', json.dumps(d['config3'])[:400]); print('3d', json.dumps(d['wstack_3d']))
print('cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/kt" -o run -- python3 bench.py --no-config3 --no-cpu-baseline \
    --steps 5 > "$OUT/kt.log" 2>&1 || { tail -5 "$OUT/kt.log"; exit 1; }
f=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+(<[^>(]*>)?)", r["Name"])
    if m: print(f'{m.group(1)[:50]:50s} {float(r["AverageNs"])/1e3:9.1f} us x {r["Calls"]}')
PY
# Optional A/B: kernel traces of library variants (name:dir ...) after it.
if [ -n "$AB" ]; then
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
fi
