#!/bin/bash
# ES GPU tests on the in-tree library, then an alternating config-2/3 A/B
# of library dirs: scripts/gpu_es_test_ab.sh OUT "dir_a dir_b" [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_es_gpu.py tests/test_es_batches_gpu.py tests/test_es_multichan_gpu.py \
    tests/test_distributed_gpu.py tests/test_baseline_configs_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
scripts/ab_lib.sh "$OUT/ab" 2 "$DIRS" --steps 20 --no-wstack "$@"
