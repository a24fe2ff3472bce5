#!/bin/bash
# fp32 row-half pipelined BPTT: numerics, A/B microbench against the two-phase kernel, fp32 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_bwdp; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "lstmf or trainer_gradients_gpu_vs_cpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 2 1 2; do
  HFREP_LSTMF_BWD=$v timeout -k 10 120 python -u scripts/bench_lstm.py --dtype float32 --batch 32768 --K 100 --only bwd --iters 20 \
      | sed "s/^/{\"ver\": $v} /" >> $O/bwd_ab.txt || { echo AB_FAIL; exit 1; }
done
cat $O/bwd_ab.txt
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --dtype float32 --batch-per-gpu 32768 > $O/bench_fp32_32k.json 2> $O/bench.err && cat $O/bench_fp32_32k.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
