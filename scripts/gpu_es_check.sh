#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5bk4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_es_gpu.py tests/test_es_multichan_gpu.py tests/test_es_batches_gpu.py tests/test_baseline_configs_gpu.py::test_config2_grid_full_size tests/test_baseline_configs_gpu.py::test_config2_degrid_full_size tests/test_baseline_configs_gpu.py::test_config3_grid_64_channels tests/test_baseline_configs_gpu.py::test_config3_degrid_64_channels tests/test_baseline_configs_gpu.py::test_wstacking_config2_geometry_vs_oracle tests/test_baseline_configs_gpu.py::test_grid_16384_fused_fft_vs_oracle tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
scripts/ab_lib.sh $OUT/ab 2 ". variants/bk_head" --steps 20
