#!/bin/bash
# Tower kernels on the GPU box: fused-tower tests, then a kernel-trace A/B of
# library variants on config 4 (grid + degrid), then (PMC=1) SQ counters of
# the default build. scripts/gpu_r4_tower.sh OUT name:libdir ...
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 \
    --timeout-method thread -k "wstack or wtower" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --warmup 1 --no-cpu-baseline" \
    scripts/kt_variants.sh "$OUT/ab" "$@" || exit $?
python3 scripts/ab_table.py "$OUT" ${@%%:*} --top 12 2>/dev/null
for spec in "$@"; do
  n=${spec%%:*}; grep -h '"metric"' "$OUT/ab/$n.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$n', d['value'], d.get('degrid', {}).get('mvis_s'))"
done
if [ "${PMC:-0}" = 1 ]; then
  BENCH=bench_wtower.py scripts/pmc_kernel.sh "$OUT/pmc" "k_tower_(dft|idft)" \
      --degrid --steps 1 --warmup 0 --no-cpu-baseline
fi
