#!/bin/bash
# Full GPU suite on the default build, then correctness + kernel-trace A/B
# of the round-4 build switches (8-wave tower kernels, 512-thread paired
# column pass).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n/full_pytest.log 2>&1 || { tail -30 gpurun_out/r4n/full_pytest.log; exit 1; }
tail -1 gpurun_out/r4n/full_pytest.log
for v in nw8 nw8w5; do
  SKA_SDP_FUNC_LIB_DIR=variants/$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wstack or wtower" > gpurun_out/r4n/pre_$v.log 2>&1 || { tail -20 gpurun_out/r4n/pre_$v.log; exit 1; }
  tail -1 gpurun_out/r4n/pre_$v.log
done
SKA_SDP_FUNC_LIB_DIR=variants/p512 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "test_es_gpu or test_es_fft_gpu or config2" > gpurun_out/r4n/pre_p512.log 2>&1 || { tail -20 gpurun_out/r4n/pre_p512.log; exit 1; }
tail -1 gpurun_out/r4n/pre_p512.log
scripts/kt_variants.sh gpurun_out/r4n/es/ab new:ska-sdp-func_amd p512:variants/p512 || exit 1
python3 scripts/ab_table.py gpurun_out/r4n/es new p512 --top 12
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --warmup 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4n/ab new:ska-sdp-func_amd nw8:variants/nw8 nw8w5:variants/nw8w5 || exit 1
python3 scripts/ab_table.py gpurun_out/r4n new nw8 nw8w5 --top 8
