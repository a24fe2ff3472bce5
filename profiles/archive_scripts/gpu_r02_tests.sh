#!/bin/bash
# full GPU test suite + the bf16 gradient-bound test with its measured errors printed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_tests; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bf16_fused" -s -q --timeout 200 --timeout-method thread 2>&1 | grep -E "bf16 rel|passed|failed" > $O/bf16_errors.txt; cat $O/bf16_errors.txt
