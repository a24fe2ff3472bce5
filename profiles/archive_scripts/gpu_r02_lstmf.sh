#!/bin/bash
# fp32 fused LSTM kernels: numerics tests, then the fp32 bench at two batch sizes + kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_lstmf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "lstmf or trainer_gradients_gpu_vs_cpu or lstm_tangent or lstm_fwd_bwd or skinny or linear" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --dtype float32 --batch-per-gpu 32768 > $O/bench_fp32_32k.json 2> $O/bench_fp32_32k.err && cat $O/bench_fp32_32k.json || { echo BENCH_FAIL; tail $O/bench_fp32_32k.err; exit 1; }
bash scripts/gpu_prof_dtype.sh r02_lstmf/prof32k float32 32768
