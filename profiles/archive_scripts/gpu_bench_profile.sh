#!/bin/bash
# usage: bash scripts/gpu_bench_profile.sh TAG "B1 B2 ..." PROF_B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-run}; BS=${2:-"16384"}; PB=${3:-16384}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for B in $BS; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch-per-gpu $B > $OUT/bench_B$B.log 2>&1 || { echo BENCH_FAIL $B; tail -30 $OUT/bench_B$B.log; exit 1; }
  tail -1 $OUT/bench_B$B.log
done
if [ "$PB" != "0" ]; then
  R=$(pwd)
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 1 --batch-per-gpu $PB > "$R/$OUT/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/$OUT/prof.log"; exit 1; }
  cd "$R" && python scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv > $OUT/prof_summary.txt && cat $OUT/prof_summary.txt
fi
