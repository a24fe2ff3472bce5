#!/bin/bash
# A/B of the LSTM recurrent kernels: lstm microbench with ab_libs/old.so vs the in-tree library,
# LSTM GPU tests, then one bench.py run.   usage: bash scripts/gpu_ab.sh TAG [BATCH]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ab}; B=${2:-16384}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "lstm" > $OUT/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for K in 100 32; do
  if [ -f ab_libs/old.so ]; then
    HFREP_NATIVE_LIB=$PWD/ab_libs/old.so timeout -k 10 200 python scripts/bench_lstm.py --batch $B --K $K --iters 10 --only fwd,tfwd,bwd,tbwd,bwd_dx,tbwd_dx > $OUT/old_K$K.log 2>&1 || { echo OLD_FAIL; tail -20 $OUT/old_K$K.log; exit 1; }
  fi
  timeout -k 10 200 python scripts/bench_lstm.py --batch $B --K $K --iters 10 --only fwd,tfwd,bwd,tbwd,bwd_dx,tbwd_dx > $OUT/new_K$K.log 2>&1 || { echo NEW_FAIL; tail -20 $OUT/new_K$K.log; exit 1; }
  echo "K=$K old / new"; grep -h '"op"' $OUT/old_K$K.log $OUT/new_K$K.log 2>/dev/null
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch-per-gpu $B > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
