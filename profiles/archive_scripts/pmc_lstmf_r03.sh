#!/bin/bash
# PMC table of the round-3 fp32 LSTM kernels (split BPTT / forward, quad + pair split weight gradients, split
# dX, exact K = 100 forward and tangent reverse): bench_lstm.py at B = 32768, K = 32 and 100, three passes
# per K (counter groups within the per-block limits), then scripts/pmc_table.py.
# usage: profiles/archive_scripts/pmc_lstmf_r03.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_r03}; mkdir -p $OUT
export TMPDIR=/tmp
OPS=fwd,fwd_notape,tfwd,bwd,tbwd,dgrad,wgrad,wgrad_tan
for K in 32 100; do
  timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 32768 --K $K --iters 5 --only $OPS > $OUT/timing_K$K.log 2>&1 || { tail $OUT/timing_K$K.log; exit 1; }
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
             "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/K$K/p$i" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 32768 --K $K --iters 2 --only $OPS > "$R/$OUT/K$K.p$i.log" 2>&1 || { echo "PMC pass K$K/$i failed"; tail -20 "$R/$OUT/K$K.p$i.log"; exit 1; }
    cd "$R"
  done
  python scripts/pmc_summary.py $OUT/K$K > $OUT/summary_K$K.txt
done
python scripts/pmc_table.py $OUT/summary_K32.txt $OUT/summary_K100.txt > $OUT/pmc_table.txt && cat $OUT/pmc_table.txt
