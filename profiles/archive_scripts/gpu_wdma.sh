#!/bin/bash
# fp32 LDS-DMA streaming weight gradient (impl 4): numerics vs fp64 / the exact kernel, then timing of
# every fp32 weight-gradient kernel at the critic's 12.6 M rows
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-wdma}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf_wgrad" -q --timeout 200 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -n 40 $OUT/tests.txt; exit 1; }
tail -n 2 $OUT/tests.txt
timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $OUT/bench_wgrad.jsonl 2>&1 \
  || { tail -n 20 $OUT/bench_wgrad.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/bench_wgrad.jsonl
if [ -f variants/wdma_il/_hfrep_native.so ]; then
  HFREP_NATIVE_LIB="$R/variants/wdma_il/_hfrep_native.so" timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf_wgrad_split_vs_exact" -q \
    --timeout 200 --timeout-method thread > $OUT/tests_il.txt 2>&1 || { tail -n 40 $OUT/tests_il.txt; exit 1; }
  tail -n 1 $OUT/tests_il.txt
  HFREP_NATIVE_LIB="$R/variants/wdma_il/_hfrep_native.so" timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 \
    > $OUT/bench_wgrad_il.jsonl 2>&1 || { tail -n 20 $OUT/bench_wgrad_il.jsonl; exit 1; }
  grep '"f32_dma"' $OUT/bench_wgrad_il.jsonl
fi
if [ -f variants/ds4_3/_hfrep_native.so ]; then
  for tag in base ds4_3; do
    if [ $tag = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$R/variants/ds4_3/_hfrep_native.so"; fi
    timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_lstmf_dgrad" -q --timeout 200 --timeout-method thread \
      > $OUT/tests_dgrad_$tag.txt 2>&1 || { tail -n 40 $OUT/tests_dgrad_$tag.txt; exit 1; }
    tail -n 1 $OUT/tests_dgrad_$tag.txt
    timeout -k 10 200 python -u scripts/bench_lstm.py --dtype float32 --batch 262144 --K 100 --iters 10 --only dgrad \
      > $OUT/dgrad_$tag.jsonl 2>&1 || { tail -n 20 $OUT/dgrad_$tag.jsonl; exit 1; }
    grep '"op"' $OUT/dgrad_$tag.jsonl
  done
  unset HFREP_NATIVE_LIB
fi
timeout -k 10 400 python -u scripts/ae_bf16_diag.py --latents 1,4,8 --seeds 1,2 > $OUT/ae_bf16_diag.jsonl 2>&1 || { tail -n 20 $OUT/ae_bf16_diag.jsonl; exit 1; }
grep '"k"' $OUT/ae_bf16_diag.jsonl
