#!/bin/bash
# Config-2 evidence in one GPU call: PMC traffic passes (each its own
# rocprofv3 run), the bench JSON line (reads the fresh traffic numbers), and
# a kernel-trace --stats summary of the same bench. Outputs under
# gpurun_out/c2/; copy the ones to keep into profiles/.
set -o pipefail
OUT=gpurun_out/c2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/pmc_traffic.sh "$OUT/pmc" --steps 3 --warmup 1 --no-cpu-baseline --no-degrid --no-config3 || exit $?
python3 scripts/pmc_traffic.py "$OUT/pmc" "$OUT/pmc_traffic.json" > /dev/null || exit $?
cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json
rm -rf "$OUT/pmc"/FETCH_SIZE "$OUT/pmc"/WRITE_SIZE
echo "== bench"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { rc=$?; tail -5 "$OUT/bench.err"; exit $rc; }
tail -1 "$OUT/bench.json"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config3 > "$OUT/kt.log" 2>&1 || { rc=$?; tail -5 "$OUT/kt.log"; exit $rc; }
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/kt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
tail -1 "$OUT/kt.log"
head -12 "$OUT/kernel_stats.csv"
