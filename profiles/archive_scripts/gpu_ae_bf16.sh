#!/bin/bash
# the bf16 autoencoder study again after the odd-K narrow-Dense fix, plus the linear-kernel tests
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_ae_bf16}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_linear" -q --timeout 200 --timeout-method thread > $OUT/tests_linear.txt 2>&1 \
  || { tail -n 30 $OUT/tests_linear.txt; exit 1; }
tail -n 1 $OUT/tests_linear.txt
timeout -k 10 600 python -u scripts/ae_study.py --out $OUT --seeds 1-30 --dtypes bfloat16 --device cuda > $OUT/study.log 2>&1 || { tail -n 20 $OUT/study.log; exit 1; }
tail -n 2 $OUT/study.log
timeout -k 10 300 python -u scripts/ae_bf16_diag.py --latents 1,3 --seeds 1 > $OUT/ae_bf16_diag.jsonl 2>&1 || { tail -n 20 $OUT/ae_bf16_diag.jsonl; exit 1; }
grep '"k"' $OUT/ae_bf16_diag.jsonl
