#!/bin/bash
# PMC passes over the default fp32 weight-gradient kernels (K = 32: split pair, K = 100: quad) at
# B = 65536 x T = 24: issue mix, MFMA busy, LDS traffic / conflicts, waits, HBM bytes.
#   bash profiles/archive_scripts/pmc_wgrad_r04.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_wgrad_r04}; mkdir -p $OUT
export TMPDIR=/tmp
for K in 32 100; do
  timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 65536 --K $K --iters 5 --only wgrad > $OUT/timing_K$K.log 2>&1 \
    || { tail $OUT/timing_K$K.log; exit 1; }
  grep op $OUT/timing_K$K.log
done
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  for K in 32 100; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p${i}_K$K" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K $K --iters 2 --only wgrad > "$R/$OUT/p${i}_K$K.log" 2>&1 \
      || { echo "PMC pass $i K=$K failed"; tail -20 "$R/$OUT/p${i}_K$K.log"; exit 1; }
  done
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
