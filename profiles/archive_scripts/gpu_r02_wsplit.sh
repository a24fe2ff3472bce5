#!/bin/bash
# split-bf16 fp32 weight gradient: numerics tests, microbench vs the exact kernel, bench at 262k
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_wsplit; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "wgrad or slice_averages or trainer_gradients_gpu_vs_cpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep "max abs err" $O/tests.log | head -20
timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $O/wgrad_bench.jsonl 2>&1 || { echo WB_FAIL; tail $O/wgrad_bench.jsonl; exit 1; }
cat $O/wgrad_bench.jsonl
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --dtype float32 > $O/bench_fp32.json 2> $O/bench.err && cat $O/bench_fp32.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
