#!/bin/bash
# Round 5 flagger: bit-exact tests on a variant library, then config-5 A/B
# (bench_flagger.py) of the in-tree build and the variant(s).
#   scripts/gpu_r5_flag.sh OUT "dir_a dir_b ..."
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2
mkdir -p "$OUT"
for d in $DIRS; do
    f=${d//\//_}
    SKA_SDP_FUNC_LIB_DIR=$d timeout -k 10 600 python -u -m pytest tests/test_flagger_gpu.py \
        -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_$f.log" 2>&1 \
        || { tail -30 "$OUT/pytest_$f.log"; exit 1; }
    echo "$d: $(tail -1 "$OUT/pytest_$f.log")"
done
for r in 1 2; do
    for d in $DIRS; do
        f=${d//\//_}
        SKA_SDP_FUNC_LIB_DIR=$d timeout -k 10 300 python -u bench_flagger.py --no-cpu-baseline \
            > "$OUT/b_${f}_$r.json" 2> "$OUT/b_${f}_$r.err" || { tail -5 "$OUT/b_${f}_$r.err"; exit 1; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" "$OUT/b_${f}_$r.json" "$d"
    done
done
