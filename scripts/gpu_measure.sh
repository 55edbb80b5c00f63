#!/bin/bash
# Round-end evidence on one GPU box: the whole GPU suite, the bench.py line
# (config 2 + config 3 + 3-D + CPU baselines), kernel-trace summaries of
# config 2 / 3-D and of config 3, the PMC traffic passes, the config-4
# (w-towers) and config-5 (flagger) lines with their traces.
#   scripts/gpu_measure.sh OUT [parts: test,es,c3,traffic,wt,flag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/measure}
PARTS=${2:-test,es,c3,traffic,wt,flag}
mkdir -p "$OUT"
stats() {   # kernel_stats.csv of a rocprofv3 output dir -> OUT/NAME
    f=$(find "$1" -name "*kernel_stats.csv" | head -1)
    cp "$f" "$OUT/$2" && find "$1" -name "*.csv" ! -name "*kernel_stats.csv" -delete
}
if [[ $PARTS == *test* ]]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread > "$OUT/pytest.log" 2>&1 \
        || { tail -40 "$OUT/pytest.log"; exit 1; }
    tail -1 "$OUT/pytest.log"
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log"
fi
if [[ $PARTS == *es* ]]; then
    timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -20 "$OUT/bench.err"; exit 1; }
    tail -c 600 "$OUT/bench.json"; echo
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/kt" -o kt -- python3 bench.py --steps 10 --warmup 3 \
        --no-cpu-baseline --no-config3 > "$OUT/kt.log" 2>&1 \
        || { tail -5 "$OUT/kt.log"; exit 1; }
    stats "$OUT/kt" bench_kernel_stats.csv || exit 1
fi
if [[ $PARTS == *c3* ]]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/c3kt" -o kt -- python3 bench.py --rows 100000 --steps 1 \
        --warmup 0 --no-cpu-baseline --no-degrid --no-wstack --c3-steps 2 \
        > "$OUT/c3kt.log" 2>&1 || { tail -5 "$OUT/c3kt.log"; exit 1; }
    stats "$OUT/c3kt" c3_kernel_stats.csv || exit 1
fi
if [[ $PARTS == *traffic* ]]; then
    scripts/pmc_traffic.sh "$OUT/traffic" --steps 3 --warmup 1 \
        --no-cpu-baseline --no-degrid --no-config3 --no-wstack || exit 1
    python3 scripts/pmc_traffic.py "$OUT/traffic" "$OUT/pmc_traffic.json" \
        > /dev/null || exit 1
    find "$OUT/traffic" -name "*.csv" ! -name "*counter_collection.csv" -delete
fi
if [[ $PARTS == *wt* ]]; then
    timeout -k 10 600 python -u bench_wtower.py --degrid > "$OUT/wtower.json" \
        2> "$OUT/wtower.err" || { tail -20 "$OUT/wtower.err"; exit 1; }
    tail -c 400 "$OUT/wtower.json"; echo
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/wkt" -o wt -- python3 bench_wtower.py --degrid --steps 1 \
        --no-cpu-baseline > "$OUT/wkt.log" 2>&1 || { tail -5 "$OUT/wkt.log"; exit 1; }
    stats "$OUT/wkt" wtower_kernel_stats.csv || exit 1
fi
if [[ $PARTS == *flag* ]]; then
    timeout -k 10 600 python -u bench_flagger.py > "$OUT/flagger.json" \
        2> "$OUT/flagger.err" || { tail -20 "$OUT/flagger.err"; exit 1; }
    tail -c 400 "$OUT/flagger.json"; echo
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/fkt" -o fl -- python3 bench_flagger.py --steps 2 --warmup 1 \
        --no-cpu-baseline > "$OUT/fkt.log" 2>&1 || { tail -5 "$OUT/fkt.log"; exit 1; }
    stats "$OUT/fkt" flagger_kernel_stats.csv || exit 1
fi
echo measure done
