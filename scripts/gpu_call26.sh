#!/bin/bash
# FFT column pass A (k_cols_a_*) counter look: HBM bytes per launch
# (FETCH_SIZE / WRITE_SIZE passes) and SQ / TCC / TCP passes, config-2
# gridding only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4c; mkdir -p $OUT
A="--steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-degrid --no-wstack"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "k_cols|k_rows" --output-format csv -d $OUT/$ctr -o pmc -- python3 bench.py $A > $OUT/$ctr.log 2>&1 || { echo "$ctr failed"; tail -5 $OUT/$ctr.log; exit 1; }
done
scripts/pmc_kernel.sh $OUT/sq "k_cols_a" $A || exit 1
echo call26 done
