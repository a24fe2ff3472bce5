#!/bin/bash
# PMC passes over the fp32 forwards (exact K = 100 lstmf_fwd, split K = 32 lstmf_fwds; primal and tangent), B = 65536
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_fwd_r04}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 65536 --K 100 --iters 5 --only fwd,tfwd > $OUT/timing.log 2>&1 && timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 65536 --K 32 --iters 5 --only fwd,tfwd >> $OUT/timing.log 2>&1 && timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K 100 --iters 3 --only fwd,tfwd >> $OUT/timing.log 2>&1 || { tail $OUT/timing.log; exit 1; }
grep op $OUT/timing.log
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  for K in 100 32; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K $K --iters 2 --only fwd,tfwd > "$R/$OUT/p$i.log" 2>&1 \
      || { echo "PMC pass $i failed"; tail -20 "$R/$OUT/p$i.log"; exit 1; }
  done
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && grep -A 24 "lstmf_fwd" $OUT/summary.txt
