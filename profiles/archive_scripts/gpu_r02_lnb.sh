#!/bin/bash
# grid-stride bf16 LayerNorm forward: numerics, then the bf16 step's kernel profile at the bench shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_lnb; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread \
    -k "layernorm or trainer_gradients or determinism or graph" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_prof_dtype.sh r02_lnb/prof262k bfloat16 262144 > /dev/null && head -26 gpurun_out/r02_lnb/prof262k/prof_summary.txt
