#!/bin/bash
# HBM traffic passes (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs,
# as they cannot share a pass) over a short gridding-only bench run.
# Usage: scripts/pmc_traffic.sh OUTDIR [bench args...]
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$ctr" -o pmc -- python3 bench.py "$@" > "$OUT/$ctr.log" 2>&1 || { rc=$?; echo "pass $ctr failed rc=$rc"; tail -5 "$OUT/$ctr.log"; exit $rc; }
done
echo traffic done
