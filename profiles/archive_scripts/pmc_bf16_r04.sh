#!/bin/bash
# PMC passes over the bf16 recurrent kernels (lstm_fwd4 / lstm_bwd3 / lstm_tbwd4), B = 65536, K = 100
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_bf16_r04}; mkdir -p $OUT
export TMPDIR=/tmp
OPS=fwd,tfwd,bwd_dx,tbwd_dx
timeout -k 10 200 python scripts/bench_lstm.py --batch 65536 --K 100 --iters 5 --only $OPS > $OUT/timing.log 2>&1 || { tail $OUT/timing.log; exit 1; }
grep op $OUT/timing.log
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_lstm.py" --batch 65536 --K 100 --iters 2 --only $OPS > "$R/$OUT/p$i.log" 2>&1 \
    || { echo "PMC pass $i failed"; tail -5 "$R/$OUT/p$i.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && echo summarised
