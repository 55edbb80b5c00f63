#!/bin/bash
# Round 5: channel-run path -- ES GPU tests, then config-3 A/B vs the
# variant in variants/base.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r5runs}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_es_runs_gpu.py tests/test_es_gpu.py \
    tests/test_es_batches_gpu.py -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
scripts/ab_c3.sh "$OUT/ab" 2 "ska-sdp-func_amd variants/base" || exit 1
