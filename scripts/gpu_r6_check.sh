#!/bin/bash
# Round 6: GPU suite (incl. the new doc / row-spectra tests), smoke, the
# default bench line and a config-2 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r6a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
    > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
tail -c 1500 "$OUT/bench.json"; echo
echo r6 check done
