#!/bin/bash
# Real-output gridding / real-input degridding FFT: ES parity tests (2-D
# paths, config 2 at full size), then A/B of SDP_ES_HERM_DEGRID on the
# config-2 bench (gridding and degridding).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/herm; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_es_gpu.py tests/test_es_fft_gpu.py tests/test_baseline_configs_gpu.py -k "not config4 and not config5" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 scripts/ab_env.sh $OUT/ab SDP_ES_HERM_DEGRID "0 1" 2 --no-config3 --steps 20
