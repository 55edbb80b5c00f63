#!/bin/bash
# Round 5: channel runs + pruned A/B switches -- ES / w-stack GPU tests, then
# config-3 A/B of the run-scatter chunk (112 default vs 128) and the base.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r5runs4}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_es_runs_gpu.py tests/test_es_gpu.py \
    tests/test_es_batches_gpu.py tests/test_es_fft_gpu.py tests/test_wstack_gpu.py \
    tests/test_dft.py -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
scripts/ab_c3.sh "$OUT/ab" 2 "ska-sdp-func_amd variants/c128 variants/base" || exit 1
