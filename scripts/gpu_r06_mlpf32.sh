#!/bin/bash
# Configs 3 / 4 fp32: rocprofv3 kernel tables of one bench iteration each (fused MLP path).
#   bash scripts/gpu_r06_mlpf32.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_mlpf32}; mkdir -p $OUT; export TMPDIR=/tmp
for M in gan wgan_gp; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt_$M" -o run -- \
    python "$R/bench.py" --model $M --dtype float32 --steps 1 --warmup 1 > "$R/$OUT/kt_$M.log" 2>&1 \
    || { cd "$R"; echo "kernel trace $M failed"; tail -5 "$OUT/kt_$M.log"; exit 1; }
  cd "$R"
  f=$(ls $OUT/kt_$M/*kernel_stats.csv $OUT/kt_$M/*/*kernel_stats.csv 2>/dev/null | head -n 1)
  python scripts/prof_summary.py "$f" 30 > $OUT/kernel_summary_$M.txt && head -n 14 $OUT/kernel_summary_$M.txt
done
