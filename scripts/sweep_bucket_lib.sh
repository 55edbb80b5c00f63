#!/bin/bash
# Like sweep_bucket.sh, with the library taken from LIBDIR (a variant):
#   scripts/sweep_bucket_lib.sh OUT LIBDIR "cv nt" ...
OUT=$1; LIB=$2; shift 2; mkdir -p $OUT
for cfg in "$@"; do
  set -- $cfg
  SKA_SDP_FUNC_LIB_DIR=$LIB SDP_ES_CHUNK_VIS=$1 SDP_ES_BUCKET_THREADS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/b_$1_$2.json 2>$OUT/b_$1_$2.err || exit $?
done
