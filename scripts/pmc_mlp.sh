#!/bin/bash
# PMC counter passes over one bench.py iteration of the fused MLP configs (one counter group per run).
#   bash scripts/pmc_mlp.sh OUTNAME [wgan_gp|gan] [bfloat16|float32]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_mlp}; M=${2:-wgan_gp}; DT=${3:-bfloat16}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/bench.py" --model $M --dtype $DT --steps 1 --warmup 1 > "$R/$OUT/p$i.log" 2>&1 || { echo "PMC pass $i failed"; tail -20 "$R/$OUT/p$i.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && python scripts/pmc_table.py $OUT/summary.txt > $OUT/table.txt; cat $OUT/table.txt; grep -A30 "mlp_gen_bwd_w" $OUT/summary.txt | head -34
