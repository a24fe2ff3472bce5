#!/bin/bash
# PMC counter passes over the LSTM recurrent-kernel microbenchmark (one counter group per run).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_lstm.py --iters 5 --only fwd,fwd_notape,tfwd,bwd,tbwd,bwd_dx,tbwd_dx > $OUT/timing.log 2>&1 || exit 1
cat $OUT/timing.log | grep op
cd /tmp
rocprofv3 -L > "$R/$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_lstm.py" --iters 2 --only fwd,fwd_notape,tfwd,bwd,tbwd,bwd_dx,tbwd_dx > "$R/$OUT/p$i.log" 2>&1 || { echo "PMC pass $i failed"; tail -20 "$R/$OUT/p$i.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
