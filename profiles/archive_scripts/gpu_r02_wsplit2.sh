#!/bin/bash
# split wgrad v2 (three column parts): numerics tests + microbench vs the exact kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_wsplit2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "wgrad_split or wgrad_large or lstmf_wgrad_fused" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $O/wgrad_bench.jsonl 2>&1 || { echo WB_FAIL; tail $O/wgrad_bench.jsonl; exit 1; }
cat $O/wgrad_bench.jsonl
