#!/bin/bash
# One GPU call's worth of round evidence: config 2 (scripts/refresh_config2.sh:
# PMC traffic, bench line, kernel-trace stats), config 4 (bench_wtower.py
# --degrid with its C/OpenMP CPU baseline, kernel-trace stats of a
# grid + degrid step) and config 5 (bench_flagger.py). Outputs under
# gpurun_out/{c2,wt,fl}; copy what is kept into profiles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/refresh_config2.sh || exit $?
OUT=gpurun_out/wt
mkdir -p "$OUT"
echo "== wtower bench"
timeout -k 10 400 python3 -u bench_wtower.py --degrid > "$OUT/bench.json" 2> "$OUT/bench.err" || { rc=$?; tail -5 "$OUT/bench.err"; exit $rc; }
tail -1 "$OUT/bench.json"
echo "== wtower kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench_wtower.py --degrid --steps 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { rc=$?; tail -5 "$OUT/kt.log"; exit $rc; }
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
head -8 "$OUT/kernel_stats.csv"
OUT=gpurun_out/fl
mkdir -p "$OUT"
echo "== flagger bench"
timeout -k 10 400 python3 -u bench_flagger.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { rc=$?; tail -5 "$OUT/bench.err"; exit $rc; }
tail -1 "$OUT/bench.json"
