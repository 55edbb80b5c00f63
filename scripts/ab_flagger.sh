#!/bin/bash
# A/B of library builds (scripts/variant_lib.sh) on the flagger bench,
# alternating runs: scripts/ab_flagger.sh OUT ROUNDS "dir_a dir_b ..." [args]
# ("." = the in-tree library).
OUT=$1; ROUNDS=$2; DIRS=$3; shift 3
cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
    for d in $DIRS; do
        lib=$d; [ "$d" = "." ] && lib=ska-sdp-func_amd
        f=${d//\//_}
        SKA_SDP_FUNC_LIB_DIR=$lib timeout -k 10 300 python3 -u bench_flagger.py \
            --no-cpu-baseline "$@" > "$OUT/f_${f}_$r.json" \
            2> "$OUT/f_${f}_$r.err" || { rc=$?; tail -5 "$OUT/f_${f}_$r.err"; exit $rc; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], 'ms', d['value'], 'Mvis/s', d['config']['flagged_fraction'])" "$OUT/f_${f}_$r.json" "$d"
    done
done
