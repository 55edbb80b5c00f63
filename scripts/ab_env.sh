#!/bin/bash
# A/B of an environment switch on the config-2 bench, alternating runs:
#   scripts/ab_env.sh OUT VAR "val_a val_b" ROUNDS [bench args]
OUT=$1; VAR=$2; VALS=$3; ROUNDS=$4; shift 4
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
    for v in $VALS; do
        f=${v//\//_}
        env "$VAR=$v" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > "$OUT/b_${f}_$r.json" 2> "$OUT/b_${f}_$r.err" || { rc=$?; tail -5 "$OUT/b_${f}_$r.err"; exit $rc; }
        python3 "$(dirname "$0")/ab_summary.py" "$OUT/b_${f}_$r.json" "$VAR=$v"
    done
done
