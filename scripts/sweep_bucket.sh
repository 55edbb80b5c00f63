#!/bin/bash
# Bench under several bucketing configurations: scripts/sweep_bucket.sh OUT "cv nt" ...
OUT=$1; shift; mkdir -p $OUT
for cfg in "$@"; do
  set -- $cfg
  SDP_ES_CHUNK_VIS=$1 SDP_ES_BUCKET_THREADS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/b_$1_$2.json 2>$OUT/b_$1_$2.err || exit $?
done
