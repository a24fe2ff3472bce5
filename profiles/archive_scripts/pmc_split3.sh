#!/bin/bash
# PMC passes over the fp32 split weight-gradient (quad) and input-gradient (LDS-staged) kernels
# (impl 3) vs the exact kernels (impl 1), B = 65536 x T = 24.  usage: scripts/pmc_split3.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_split3}; mkdir -p $OUT
export TMPDIR=/tmp
for impl in 3 1; do
  for K in 100 32; do
    export HFREP_LSTMF_WGRAD=$impl HFREP_LSTMF_DGRAD_IMPL=$impl
    timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 65536 --K $K --iters 5 --only wgrad_tan,dgrad \
      > $OUT/timing_i${impl}_k$K.log 2>&1 || { tail $OUT/timing_i${impl}_k$K.log; exit 1; }
    grep op $OUT/timing_i${impl}_k$K.log
  done
done
export HFREP_LSTMF_WGRAD=3 HFREP_LSTMF_DGRAD_IMPL=3
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K 100 --iters 2 --only wgrad_tan,dgrad > "$R/$OUT/p$i.log" 2>&1 || { echo "PMC pass $i failed"; tail -20 "$R/$OUT/p$i.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
