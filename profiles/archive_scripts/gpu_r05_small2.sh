#!/bin/bash
# Round-5 small-batch pass 2: weight gradients on side stream 2 (HFREP_WGRAD_SIDE) -- the bitwise
# concurrency test, bench_small A/B (side stream on / off), and a kernel trace of the B = 32 iteration.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_small2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_runtime.py -k concurrent \
  > $OUT/tests_concurrent.txt 2>&1 || { tail -n 30 $OUT/tests_concurrent.txt; exit 1; }
tail -n 3 $OUT/tests_concurrent.txt
timeout -k 10 300 python -u scripts/bench_small.py --iters 300 > $OUT/small_wside1.jsonl 2>&1 || { tail -n 20 $OUT/small_wside1.jsonl; exit 1; }
HFREP_WGRAD_SIDE=0 timeout -k 10 300 python -u scripts/bench_small.py --iters 300 > $OUT/small_wside0.jsonl 2>&1 || { tail -n 20 $OUT/small_wside0.jsonl; exit 1; }
grep -h '"ms' $OUT/small_wside*.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_f32 -o run -- python3 scripts/bench_small.py --iters 20 --dtypes float32 > $OUT/prof_f32.log 2>&1 || { tail -n 20 $OUT/prof_f32.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bf16 -o run -- python3 scripts/bench_small.py --iters 20 --dtypes bfloat16 > $OUT/prof_bf16.log 2>&1 || { tail -n 20 $OUT/prof_bf16.log; exit 1; }
echo done
