#!/bin/bash
# A/B of k_tower_idft variants: parity tests on one variant, bench on all.
# The variants are library builds made beforehand with scripts/variant_lib.sh
# (round 3: base = the HEAD source via REPLACES=..., c16w5 / c16w6 / c32w4 =
# -DSDP_IDFT_CAP=16|32 -DTOWER_IDFT_WAVES=5|6|4), e.g.
#   scripts/variant_lib.sh c16w6 csrc/grid_data/sdp_grid_wstack_wtower.hip \
#       -DSDP_IDFT_CAP=16 -DTOWER_IDFT_WAVES=6
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wt_ab; mkdir -p $OUT
SKA_SDP_FUNC_LIB_DIR=variants/c16w5 timeout -k 10 300 python -u -m pytest tests/test_wstack_gpu.py tests/test_wtower_vla_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do for v in base c16w5 c16w6 c32w4; do
  SKA_SDP_FUNC_LIB_DIR=variants/$v timeout -k 10 200 python -u bench_wtower.py --degrid --no-cpu-baseline --steps 2 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -5 $OUT/$v.$r.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/$v.$r.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['avg_launch_ms'], d['degrid']['mvis_s'], d['degrid']['roofline']['avg_launch_ms'])"
done; done
