#!/bin/bash
# Run one probe script (and optionally a pytest selection) on the GPU box.
#   scripts/gpu_probe.sh OUT probe.py [pytest args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; PROBE=$2; shift 2
mkdir -p "$OUT"
if [ "$PROBE" != "-" ]; then
    timeout -k 10 300 python -u "$PROBE" > "$OUT/probe.log" 2>&1 \
        || { tail -30 "$OUT/probe.log"; exit 1; }
    cat "$OUT/probe.log"
fi
if [ $# -gt 0 ]; then
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 \
        --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1 \
        || { tail -40 "$OUT/pytest.log"; exit 1; }
    tail -3 "$OUT/pytest.log"
fi
echo probe done
