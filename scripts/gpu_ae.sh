#!/bin/bash
# Autoencoder study on the GPU (BASELINE config 2): the fused-fit tests, then 30 seeds x {fp32, bf16} x
# {real, generator-augmented} latent sweeps k = 1..21 in one process (every fit = one csrc/ae.hip launch),
# then a kernel trace of one seed's sweeps (which kernels an AE fit runs).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_ae}; mkdir -p $OUT
SEEDS=${2:-1-30}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -q --timeout 200 --timeout-method thread > $OUT/tests_ae.txt 2>&1 \
  || { tail -n 30 $OUT/tests_ae.txt; exit 1; }
tail -n 2 $OUT/tests_ae.txt
timeout -k 10 900 python -u scripts/ae_study.py --out $OUT --seeds $SEEDS --dtypes float32,bfloat16 --device cuda > $OUT/study.log 2>&1 \
  || { tail -n 20 $OUT/study.log; exit 1; }
tail -n 3 $OUT/study.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- python "$R/scripts/ae_study.py" --out /tmp/ae_prof --seeds 1-1 --dtypes float32,bfloat16 --device cuda > "$R/$OUT/prof.log" 2>&1 || { tail "$R/$OUT/prof.log"; exit 1; }
cd "$R" && python scripts/prof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 30 > $OUT/kernel_summary.txt 2>&1; head -20 $OUT/kernel_summary.txt
