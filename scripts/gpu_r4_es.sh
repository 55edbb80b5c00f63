#!/bin/bash
# ES path on the GPU box: the ES parity tests (2-D / 3-D, batches, fused
# FFT, baseline configs 2/3), a kernel-trace A/B of library variants and
# (PMC=1) SQ counters of the tile kernels.  scripts/gpu_r4_es.sh OUT name:dir ...
set -o pipefail
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "test_es_gpu or test_es_fft_gpu or batches or wstacking or config_2 or config_3 or config2 or config3" \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
scripts/kt_variants.sh "$OUT/ab" "$@" || exit 1
python3 scripts/ab_table.py "$OUT" ${@%%:*} --top 30
if [ "${PMC:-0}" = 1 ]; then
  scripts/pmc_kernel.sh "$OUT/pmc" "k_scatter_tab|k_gather_win|k_bucket" \
      --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-wstack
fi
