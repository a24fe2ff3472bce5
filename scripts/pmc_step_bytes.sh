#!/bin/bash
# HBM byte budget of whole training iterations: TCC_EA0 read / write requests of every dispatch of
# bench.py (1 warmup + 1 timed iteration at the bench shape), summed per kernel and per iteration.
#   bash scripts/pmc_step_bytes.sh OUTNAME [bfloat16|float32 ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-step_bytes}; shift; mkdir -p $OUT
export TMPDIR=/tmp
for dt in ${@:-bfloat16}; do
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      --kernel-trace --output-format csv -d "$R/$OUT/$dt" -o run -- python "$R/bench.py" --dtype $dt --steps 1 --warmup 1 \
      > "$R/$OUT/$dt.log" 2>&1 || { echo "PMC pass $dt failed"; tail -5 "$R/$OUT/$dt.log"; exit 1; }
  cd "$R" && python scripts/step_bytes_summary.py $OUT/$dt 2 > $OUT/summary_$dt.txt && head -25 $OUT/summary_$dt.txt
done
