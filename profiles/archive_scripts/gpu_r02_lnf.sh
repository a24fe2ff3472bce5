#!/bin/bash
# fp32 LayerNorm forward (16-byte half-wave rows): numerics + fp32 bench + kernel profile at 32k
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_lnf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "layernorm or trainer_gradients or lstmf" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_prof_dtype.sh r02_lnf/prof32k float32 32768 > /dev/null && head -24 gpurun_out/r02_lnf/prof32k/prof_summary.txt
rm -f gpurun_out/r02_lnf/tbwd_ab.txt
for v in 1 2 1 2; do
  HFREP_LSTMF_TBWD=$v timeout -k 10 120 python -u scripts/bench_lstm.py --dtype float32 --batch 32768 --K 100 --only tbwd --iters 20 \
      | sed "s/^/{\"ver\": $v} /" >> gpurun_out/r02_lnf/tbwd_ab.txt || { echo AB_FAIL; exit 1; }
done
cat gpurun_out/r02_lnf/tbwd_ab.txt
