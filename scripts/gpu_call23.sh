#!/bin/bash
# Where k_tower_idft's LDS bank conflicts come from: SQ counters of
# diagnostic builds that drop one LDS access class each (results wrong).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4r
for v in ska-sdp-func_amd variants/noku variants/nokv variants/noacc; do
  n=$(basename $v)
  SKA_SDP_FUNC_LIB_DIR=$v timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex "k_tower_idft" --output-format csv -d gpurun_out/r4r/$n -o pmc -- python3 bench_wtower.py --degrid --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4r/$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/r4r/$n.log; }
done
echo diag done
