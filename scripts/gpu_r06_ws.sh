#!/bin/bash
# fp32 split-bf16 weight gradient (gemm.hip wgrad_f32s_kernel): the wgrad / linear kernel tests, the fused
# MLP tests, fp32 config 3 / 4 benches and their kernel tables.
#   bash scripts/gpu_r06_ws.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_ws}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or linear" -x -q --timeout 240 \
  --timeout-method thread > $OUT/tests_k.txt 2>&1
rc=$?; tail -n 2 $OUT/tests_k.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 240 --timeout-method thread \
  > $OUT/tests.txt 2>&1
rc=$?; tail -n 2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for M in wgan_gp gan; do
  timeout -k 10 200 python bench.py --model $M --dtype float32 --steps 10 --warmup 2 > $OUT/${M}_f32.json \
    2> $OUT/${M}_f32.err || { tail $OUT/${M}_f32.err; exit 1; }
done
bash scripts/gpu_r06_mlpf32.sh ${1:-r06_ws}
