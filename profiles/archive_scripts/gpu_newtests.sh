#!/bin/bash
# the round-3 GPU tests added last: large-batch bf16 tangent-reverse determinism + the head-adjoint test
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-newtests}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bitwise_large_batch or head_adjoint_in_kernel" -v --timeout 200 \
  --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/tests.txt | tail -6
