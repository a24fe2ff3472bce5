#!/bin/bash
# Kernel numerics for the split fp32 kernels, then timing + PMC of the split forward (K = 32, tape)
# and the LDS-staged input gradient at B = 262144 x T = 24.  usage: scripts/pmc_fwd_dgrad.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-pmc_fwd_dgrad}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf_dgrad or split_forward or gp_coef" -q --timeout 200 \
  --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
tail -n 1 $OUT/tests.txt
timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K 32 --iters 5 --only fwd,fwd_notape,tfwd \
  > $OUT/timing_fwd.log 2>&1 || { tail $OUT/timing_fwd.log; exit 1; }
timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K 100 --iters 5 --only dgrad,fwd \
  > $OUT/timing_k100.log 2>&1 || { tail $OUT/timing_k100.log; exit 1; }
grep -h op $OUT/timing_fwd.log $OUT/timing_k100.log
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/p$i" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K 32 --iters 1 --only fwd > "$R/$OUT/p$i.log" 2>&1 || { echo "PMC pass $i failed"; tail -20 "$R/$OUT/p$i.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && grep -A20 "lstmf_fwds" $OUT/summary.txt
