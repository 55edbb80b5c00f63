#!/bin/bash
# SQ + cache PMC passes for kernels matching REGEX over a short bench run:
#   [BENCH=bench_flagger.py] scripts/pmc_kernel.sh OUT REGEX [bench args]
OUT=$1; RE=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"; i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RE" --output-format csv -d "$OUT/pass$i" -o pmc -- python3 "${BENCH:-bench.py}" "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/pass$i.log"; }
done
echo pmc done
