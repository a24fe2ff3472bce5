#!/bin/bash
# split-bf16 fp32 input gradient: tests, microbench vs exact / hipBLASLt, bench at 262k
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_dsplit; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "dgrad or slice_averages or trainer_gradients_gpu_vs_cpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/dgrad_fp32_bench.py 786432 6291456 > $O/dgrad_bench.jsonl 2>&1 || { echo DB_FAIL; tail $O/dgrad_bench.jsonl; exit 1; }
cat $O/dgrad_bench.jsonl
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --dtype float32 > $O/bench_fp32.json 2> $O/bench.err && cat $O/bench_fp32.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
