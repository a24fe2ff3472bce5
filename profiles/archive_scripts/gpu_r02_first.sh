#!/bin/bash
# Round-2 first GPU pass: GPU tests, bf16 bench, fp32 bench (current fp32 path) at two batch sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_first; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > $O/bench_bf16.json 2> $O/bench_bf16.err && cat $O/bench_bf16.json
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --dtype float32 --batch-per-gpu 32768 > $O/bench_fp32_32k.json 2> $O/bench_fp32_32k.err && cat $O/bench_fp32_32k.json
