#!/bin/bash
# SQ-only PMC passes: scripts/pmc_sq.sh OUT REGEX bench args
OUT=$1; RE=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"; i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RE" --output-format csv -d "$OUT/pass$i" -o pmc -- python3 ${BENCH:-bench.py} "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
echo pmc done
