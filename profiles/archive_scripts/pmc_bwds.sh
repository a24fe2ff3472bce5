#!/bin/bash
# fp32 BPTT kernels: timing of the exact (impl 1 / 2) and split-recurrent (impl 3) BPTT at B = 262144 x
# T = 24 plus PMC passes over impl 3 and impl 2.  usage: scripts/pmc_bwds.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_bwds}; mkdir -p $OUT
export TMPDIR=/tmp
for impl in 3 2 1; do
  HFREP_LSTMF_BWD=$impl timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K 32 --iters 5 \
    --only bwd,tbwd > $OUT/timing_i$impl.log 2>&1 || { tail $OUT/timing_i$impl.log; exit 1; }
  sed "s/^/impl $impl /" $OUT/timing_i$impl.log | grep op
done
cd /tmp
for impl in 3 2; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    HFREP_LSTMF_BWD=$impl timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p${impl}_$i" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 262144 --K 32 --iters 1 --only bwd > "$R/$OUT/p${impl}_$i.log" 2>&1 || { echo "PMC pass $impl/$i failed"; tail -20 "$R/$OUT/p${impl}_$i.log"; exit 1; }
  done
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && grep -A20 "lstmf_bwd" $OUT/summary.txt
