#!/bin/bash
# PMC passes over the bf16 LSTM weight gradient (lstm_wgrad3, LDS-DMA streaming) at the bench shape
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_wgrad3_r04}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_wgrad.py --dtype bfloat16 --batch 262144 --iters 5 > $OUT/timing.log 2>&1 || { tail $OUT/timing.log; exit 1; }
grep kernel $OUT/timing.log
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_wgrad.py" --dtype bfloat16 --batch 65536 --iters 2 > "$R/$OUT/p$i.log" 2>&1 \
    || { echo "PMC pass $i failed"; tail -5 "$R/$OUT/p$i.log"; break; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && grep -A 30 "wgrad3" $OUT/summary.txt
