#!/bin/bash
# W-towers: the w-stack / VLA / doc GPU tests, the config-4 line (grid +
# degrid, no CPU baseline) and its kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/wt}
mkdir -p "$OUT"
TESTS=${2:-tests/test_wstack_gpu.py tests/test_wtower_vla_gpu.py tests/test_integration_docs.py tests/test_wtower_gpu.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
    --timeout-method thread $TESTS \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 python -u bench_wtower.py --degrid --no-cpu-baseline \
    > "$OUT/wtower.json" 2> "$OUT/wtower.err" || { tail -20 "$OUT/wtower.err"; exit 1; }
tail -c 600 "$OUT/wtower.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/wkt" -o wt -- python3 bench_wtower.py --degrid --steps 1 \
    --no-cpu-baseline > "$OUT/wkt.log" 2>&1 || { tail -5 "$OUT/wkt.log"; exit 1; }
f=$(find "$OUT/wkt" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/wtower_kernel_stats.csv" && find "$OUT/wkt" -name "*.csv" ! -name "*kernel_stats.csv" -delete
echo wt done
