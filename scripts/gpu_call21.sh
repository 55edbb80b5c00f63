#!/bin/bash
# s_setprio around the matrix-op loops: ES scatter (prio) and tower kernels
# (tprio), correctness then kernel-trace A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p
SKA_SDP_FUNC_LIB_DIR=variants/prio timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "test_es_gpu or config2" > gpurun_out/r4p/pre_prio.log 2>&1 || { tail -20 gpurun_out/r4p/pre_prio.log; exit 1; }
tail -1 gpurun_out/r4p/pre_prio.log
SKA_SDP_FUNC_LIB_DIR=variants/tprio timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wstack or wtower" > gpurun_out/r4p/pre_tprio.log 2>&1 || { tail -20 gpurun_out/r4p/pre_tprio.log; exit 1; }
tail -1 gpurun_out/r4p/pre_tprio.log
scripts/kt_variants.sh gpurun_out/r4p/es/ab new:ska-sdp-func_amd prio:variants/prio new2:ska-sdp-func_amd prio2:variants/prio || exit 1
python3 scripts/ab_table.py gpurun_out/r4p/es new prio new2 prio2 --top 5
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --warmup 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4p/ab new:ska-sdp-func_amd tprio:variants/tprio || exit 1
python3 scripts/ab_table.py gpurun_out/r4p new tprio --top 4
