#!/bin/bash
# bf16 DX + GEN tangent-reverse determinism (profiles/r02_det, profiles/r03_race): the variant library
# variants/dxgen (built with -DHFREP_TBWD_DXGEN=1: the fused-dX + generated-head-adjoint tangent reverse
# dispatched) through the bitwise run-to-run script at small and bench-like batches, and the bf16 LSTM
# kernel tests on that library.
# usage: scripts/gpu_race.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-race}; mkdir -p $OUT
export HFREP_NATIVE_LIB=$R/variants/dxgen/_hfrep_native.so HFREP_TBWD_DXGEN=1
timeout -k 10 200 python scripts/dbg_determinism.py 1 3 > $OUT/det_small.txt 2>&1 || { tail $OUT/det_small.txt; exit 1; }
grep -c "False" $OUT/det_small.txt; grep False $OUT/det_small.txt | head
timeout -k 10 300 python scripts/dbg_determinism.py 128 1 > $OUT/det_large.txt 2>&1 || { tail $OUT/det_large.txt; exit 1; }
grep -c "False" $OUT/det_large.txt; grep False $OUT/det_large.txt | head
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstm2 or tbwd or tangent or gp" -q --timeout 200 --timeout-method thread \
  > $OUT/tests_variant.txt 2>&1 || { tail -n 30 $OUT/tests_variant.txt; exit 1; }
tail -n 2 $OUT/tests_variant.txt
