#!/bin/bash
# A/B of an env-selected kernel variant inside one library build.
#   usage: bash scripts/gpu_bwd_ab.sh TAG ENVVAR VALUE OPS [BATCH]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; EV=$2; VAL=$3; OPS=$4; B=${5:-16384}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for K in 100 32; do
  env $EV=$VAL timeout -k 10 200 python scripts/bench_lstm.py --batch $B --K $K --iters 10 --only $OPS > $OUT/old_K$K.log 2>&1 || { tail -20 $OUT/old_K$K.log; exit 1; }
  timeout -k 10 200 python scripts/bench_lstm.py --batch $B --K $K --iters 10 --only $OPS > $OUT/new_K$K.log 2>&1 || { tail -20 $OUT/new_K$K.log; exit 1; }
  echo "K=$K $EV=$VAL / default"; grep -h '"op"' $OUT/old_K$K.log $OUT/new_K$K.log
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch-per-gpu $B > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
