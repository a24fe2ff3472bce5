#!/bin/bash
# role-split reverse kernels with one-group operand lookahead: numerics + timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_pref; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "lstmf or trainer_gradients_gpu_vs_cpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python -u scripts/bench_lstm.py --dtype float32 --batch 32768 --K 100 --only bwd,tbwd --iters 20 >> $O/timing.txt || { echo T_FAIL; exit 1; }
done
cat $O/timing.txt
