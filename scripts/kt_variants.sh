#!/bin/bash
# Kernel-trace A/B of library variants (scripts/variant_lib.sh) on the
# config-2 bench: scripts/kt_variants.sh OUT name:libdir[:VAR=value] ...
# (BENCH / BENCH_ARGS select another bench script and its arguments.)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r n d e <<< "$spec"
  env SKA_SDP_FUNC_LIB_DIR="$d" $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- python3 ${BENCH:-bench.py} ${BENCH_ARGS:---no-config3 --no-cpu-baseline --steps 10} > "$OUT/$n.log" 2>&1 || exit $?
done
