#!/bin/bash
# Padded tower twiddle table (default) vs unpadded: tower tests + A/B + SQ
# LDS-conflict counters.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4q
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wstack or wtower" > gpurun_out/r4q/pytest.log 2>&1 || { tail -20 gpurun_out/r4q/pytest.log; exit 1; }
tail -1 gpurun_out/r4q/pytest.log
BENCH=bench_wtower.py BENCH_ARGS="--degrid --steps 1 --warmup 1 --no-cpu-baseline" \
    scripts/kt_variants.sh gpurun_out/r4q/ab new:ska-sdp-func_amd nopad:variants/nopad new2:ska-sdp-func_amd || exit 1
python3 scripts/ab_table.py gpurun_out/r4q new nopad new2 --top 4
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_tower_(dft|idft)" --output-format csv -d gpurun_out/r4q/pmc -o pmc -- python3 bench_wtower.py --degrid --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4q/pmc.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/r4q/pmc 2>&1 | tail -16
