#!/bin/bash
# A/B of library variants (scripts/variant_lib.sh) on the ES bench after
# the ES GPU tests on each variant: scripts/gpu_ab_call.sh OUT "dirs"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; DIRS=$2
mkdir -p $OUT
for d in $DIRS; do
    [ "$d" = "." ] && continue
    SKA_SDP_FUNC_LIB_DIR=$d timeout -k 10 600 python -u -m pytest tests/test_es_gpu.py tests/test_es_multichan_gpu.py tests/test_es_batches_gpu.py tests/test_baseline_configs_gpu.py::test_config2_grid_full_size tests/test_baseline_configs_gpu.py::test_config3_grid_64_channels tests/test_baseline_configs_gpu.py::test_wstacking_config2_geometry_vs_oracle tests/test_baseline_configs_gpu.py::test_grid_16384_fused_fft_vs_oracle -x -q --timeout 300 --timeout-method thread > $OUT/t_${d//\//_}.log 2>&1 || { tail -30 $OUT/t_${d//\//_}.log; exit 1; }
    echo "$d $(tail -1 $OUT/t_${d//\//_}.log)"
done
scripts/ab_lib.sh $OUT/ab 2 "$DIRS" --steps 20
