#!/bin/bash
# PMC passes over bench_flagger.py (small B). Usage: scripts/pmc_flagger.sh OUTDIR [bench args]
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"; i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_flagger" --output-format csv -d "$OUT/pass$i" -o pmc -- python3 bench_flagger.py "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
echo pmc done
