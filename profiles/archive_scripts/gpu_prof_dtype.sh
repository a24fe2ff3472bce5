#!/bin/bash
# rocprofv3 kernel stats of the training step at one dtype / batch.  usage: gpu_prof_dtype.sh TAG DTYPE B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; DT=$2; B=$3
R=$(pwd); OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 1 --batch-per-gpu $B --dtype $DT > "$R/$OUT/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/$OUT/prof.log"; exit 1; }
cd "$R" && F=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1) && python scripts/prof_summary.py $F 30 > $OUT/prof_summary.txt && cat $OUT/prof_summary.txt
