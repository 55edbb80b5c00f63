#!/bin/bash
# Flagger evidence on one GPU box: its GPU tests (incl. the full config-5
# shape), the config-5 bench line and a kernel trace of it.
#   scripts/gpu_flagger_check.sh OUT
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/flagger}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_flagger_gpu.py \
    "tests/test_baseline_configs_gpu.py::test_config5_flagger_full_size" \
    -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python -u bench_flagger.py > "$OUT/flagger.json" \
    2> "$OUT/flagger.err" || { tail -20 "$OUT/flagger.err"; exit 1; }
tail -c 300 "$OUT/flagger.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/fkt" -o fkt -- python3 bench_flagger.py --steps 3 --warmup 1 \
    --no-cpu-baseline > "$OUT/fkt.log" 2>&1 || { tail -5 "$OUT/fkt.log"; exit 1; }
f=$(find "$OUT/fkt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/flagger_kernel_stats.csv" && find "$OUT/fkt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo flagger check done
