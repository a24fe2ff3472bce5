#!/bin/bash
# Round-5 PMC passes over the final recurrent kernels (bench_lstm.py ops at B = 131072, K = 100,
# act = tanh), bf16 and fp32: MFMA busy, VALU per MFMA, LDS bank conflicts, wait cycles.  One counter
# group per rocprofv3 run; usage: bash scripts/gpu_r05_pmc.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_pmc}; mkdir -p $OUT
export TMPDIR=/tmp
OPS="fwd,fwd_notape,tfwd,bwd,bwd_dx,tbwd,tbwd_dx,wgrad"
for dt in bfloat16 float32; do
  ARGS="--batch 131072 --K 100 --act 2 --dtype $dt"
  D=$OUT/$dt; mkdir -p $D
  timeout -k 10 240 python -u scripts/bench_lstm.py $ARGS --iters 5 --only $OPS > $D/timing.jsonl 2> $D/timing.err || { tail -20 $D/timing.err; exit 1; }
  cat $D/timing.jsonl
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    echo "$dt pass $i"
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$R/$D/p$i" -o run -- python3 "$R/scripts/bench_lstm.py" $ARGS --iters 2 --only $OPS > "$R/$D/p$i.log" 2>&1) || { echo "PMC pass $i failed"; tail -20 "$R/$D/p$i.log"; exit 1; }
  done
  python scripts/pmc_summary.py $D > $D/summary.txt && python scripts/pmc_table.py $D/summary.txt > $D/table.txt && cat $D/table.txt
done
