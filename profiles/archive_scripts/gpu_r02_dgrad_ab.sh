#!/bin/bash
# fp32 headline step with the native LSTM dgrad (default) vs hipBLASLt (HFREP_LSTMF_DGRAD=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r02_dgrad_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "lstmf or trainer_gradients_gpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1; do
  HFREP_LSTMF_DGRAD=$v timeout -k 10 200 python -u bench.py --dtype float32 --steps 4 --warmup 2 > $O/bench_dgrad$v.json 2> $O/bench_dgrad$v.err \
      || { echo BENCH_FAIL; tail $O/bench_dgrad$v.err; exit 1; }
  echo "dgrad=$v $(cat $O/bench_dgrad$v.json)"
done
