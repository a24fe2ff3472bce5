#!/bin/bash
# Row-half pipelined split forward (impl 3) vs the split forward (impl 2): numerics test, then timing of
# the forward / no-tape forward at B = 262144 x T = 24 (K = 32, 36), impl 2 and 3 alternating.
# usage: scripts/gpu_fwdp.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-fwdp}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split_forward" -q --timeout 200 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -n 40 $OUT/tests.txt; exit 1; }
tail -n 1 $OUT/tests.txt
for rep in 1 2; do
  for impl in 2 3; do
    for K in 32 36; do
      HFREP_LSTMF_FWD=$impl timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K $K --iters 5 \
        --only fwd,fwd_notape > $OUT/t_${impl}_${K}_$rep.log 2>&1 || { tail $OUT/t_${impl}_${K}_$rep.log; exit 1; }
      grep op $OUT/t_${impl}_${K}_$rep.log | sed "s/^/impl $impl /"
    done
  done
done
